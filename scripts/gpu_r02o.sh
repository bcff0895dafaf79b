set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02o
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_slab.py -q -rf --timeout 300 --timeout-method thread > gpurun_out/r02o/multi.log 2>&1; echo "multi rc=$?"
echo all-done
