set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02zb
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit 1
echo all-done
