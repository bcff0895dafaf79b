set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02i
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -q -s -rf --timeout 300 --timeout-method thread -k "c1_exact or 65536 or 16384 or chunked or precond_1d" > gpurun_out/r02i/t1d.log 2>&1; echo "t1d rc=$?"
timeout -k 10 300 python bench.py --config c1 --steps 50 --warmup 5 --no-pmc --no-cpu-baseline > gpurun_out/r02i/bench_c1.json 2>gpurun_out/r02i/bench_c1.err || exit 1
PDHG_FS16=0 timeout -k 10 300 python bench.py --config c1 --steps 50 --warmup 5 --no-pmc --no-cpu-baseline > gpurun_out/r02i/bench_c1_wide.json 2>/dev/null || exit 1
bash scripts/profile.sh c1 r02_c1f16 || exit 1
echo all-done
