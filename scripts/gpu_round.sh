set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_slab.py tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_slab.log 2>&1 || exit 1
timeout -k 10 300 python scripts/slab_local_bench.py tslab c3 8 3 > gpurun_out/slab8.json 2> gpurun_out/slab8.err || exit 1
