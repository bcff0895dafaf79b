set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02w
mkdir -p $OUT
timeout -k 10 900 bash scripts/profile.sh c3 r02final > $OUT/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit 1
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 3 --no-pmc > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 1
echo all-done
