set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02r
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_slab.py -q -rf --timeout 300 --timeout-method thread -k "dma or c3_ws or c3_fr or 4096" > gpurun_out/r02r/t.log 2>&1; echo "t rc=$?"
timeout -k 10 400 python bench.py --config c3 --steps 5 --warmup 1 --no-pmc --no-cpu-baseline --no-probe > gpurun_out/r02r/bench_c3.json 2>/dev/null || exit 1
PDHG_XT_DMA=0 timeout -k 10 400 python bench.py --config c3 --steps 5 --warmup 1 --no-pmc --no-cpu-baseline --no-probe > gpurun_out/r02r/bench_c3_batch.json 2>/dev/null || exit 1
echo all-done
