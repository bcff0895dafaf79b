set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02j
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -q -s -rf --timeout 300 --timeout-method thread -k "c1_exact or 65536 or 16384 or chunked or precond_1d or e1d1 or e2d1" > gpurun_out/r02j/t1d.log 2>&1; echo "t1d rc=$?"
for G in 16 4 8; do
PDHG_F16_GROUP=$G timeout -k 10 300 python bench.py --config c1 --steps 50 --warmup 5 --no-pmc --no-cpu-baseline > gpurun_out/r02j/bench_c1_g$G.json 2>gpurun_out/r02j/bench_c1_g$G.err || exit 1
done
echo all-done
