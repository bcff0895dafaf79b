# round 2: the whole GPU suite at the new defaults (minus the fixture still being generated)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02f
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -s -rf --timeout 300 --timeout-method thread -k "not c3_fr_4096x256" > gpurun_out/r02f/gpu_suite.log 2>&1; echo "suite rc=$?"
grep -E "^(CFG|ONESTEP)" gpurun_out/r02f/gpu_suite.log > gpurun_out/r02f/cfg_lines.log || true

timeout -k 10 300 python bench.py --config c1 --steps 50 --warmup 5 --no-pmc --no-cpu-baseline > gpurun_out/r02f/bench_c1.json 2>/dev/null || exit 1
PDHG_THOMAS_CHUNK=0 timeout -k 10 300 python bench.py --config c1 --steps 50 --warmup 5 --no-pmc --no-cpu-baseline > gpurun_out/r02f/bench_c1_old.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-pmc --no-cpu-baseline > gpurun_out/r02f/bench_c3.json 2>/dev/null || exit 1
echo all-done
