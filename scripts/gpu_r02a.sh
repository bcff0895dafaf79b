# round 2, first GPU pass: config-instantiation parity, smoke, C3 bench (+PMC, CPU baseline), gloo N=2 launcher
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -v -s --timeout 300 --timeout-method thread -k "not c2_x2048" > gpurun_out/r02a_configs.log 2>&1; echo "configs rc=$?"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02a_smoke.log 2>&1 || exit 1
timeout -k 10 900 python bench.py > gpurun_out/r02a_bench_c3.json 2> gpurun_out/r02a_bench_c3.err || exit 1
PDHG_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --config c2 --steps 3 --warmup 1 > gpurun_out/r02a_bench_c2_gloo2.json 2> gpurun_out/r02a_bench_c2_gloo2.err || exit 1
echo all-done
