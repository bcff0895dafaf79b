set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_xslab.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_xs.log 2>&1 || exit 1
