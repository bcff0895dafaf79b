set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02e
run() { timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-pmc --no-cpu-baseline --no-probe > gpurun_out/r02e/$1.json 2>/dev/null; }
PDHG_XT_BATCH=1 run b4 || exit 1
PDHG_XT_BATCH=0 run ws || exit 1
PDHG_XT_BATCH=1 PDHG_DBG=3 run b4_dbg3 || exit 1
PDHG_XT_BATCH=1 run b4b || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -q --timeout 300 --timeout-method thread -k "batched" > gpurun_out/r02e/batched.log 2>&1; echo "batched rc=$?"
echo all-done
