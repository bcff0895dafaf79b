set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 bash scripts/profile.sh c3 r01f > gpurun_out/prof_f.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python bench.py > gpurun_out/bench_c3_full.json 2> gpurun_out/bench_full.err || exit 1
timeout -k 10 300 python bench.py --config c1 --steps 50 --warmup 5 --no-pmc > gpurun_out/b_c1.json 2>/dev/null || exit 1
