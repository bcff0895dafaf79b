set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02s
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/r02s/t.log 2>&1; echo "t rc=$?"
timeout -k 10 400 python bench.py --config c3 --steps 5 --warmup 1 --no-pmc --no-cpu-baseline --no-probe > gpurun_out/r02s/bench_c3.json 2>gpurun_out/r02s/bench_c3.err || exit 1
echo all-done
