set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02l
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -q -s -rf --timeout 300 --timeout-method thread -k "dma or c3_ws_T200 or c3_fr" > gpurun_out/r02l/tdma.log 2>&1; echo "tdma rc=$?"
PDHG_XT_DMA=1 timeout -k 10 400 python bench.py --config c3 --steps 5 --warmup 1 --no-pmc --no-cpu-baseline --no-probe > gpurun_out/r02l/bench_c3_dma.json 2>gpurun_out/r02l/bench_c3_dma.err || exit 1
timeout -k 10 400 python bench.py --config c3 --steps 5 --warmup 1 --no-pmc --no-cpu-baseline --no-probe > gpurun_out/r02l/bench_c3.json 2>/dev/null || exit 1
echo all-done
