set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02q
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -rf --timeout 300 --timeout-method thread -k "dual or iterate or config or one_step" > gpurun_out/r02q/t.log 2>&1; echo "t rc=$?"
timeout -k 10 400 python bench.py --config c3 --steps 5 --warmup 1 --no-pmc --no-cpu-baseline --no-probe > gpurun_out/r02q/bench_c3.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --config c1 --steps 50 --warmup 5 --no-pmc --no-cpu-baseline --no-probe > gpurun_out/r02q/bench_c1.json 2>/dev/null || exit 1
echo all-done
