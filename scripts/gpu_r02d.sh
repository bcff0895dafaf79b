# round 2: batched x transform variants (debug switches, prefetch depth), C3 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02d
run() { timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-pmc --no-cpu-baseline --no-probe > gpurun_out/r02d/$1.json 2>/dev/null; }
PDHG_XT_BATCH=0 run ws || exit 1
PDHG_XT_BATCH=1 run b0 || exit 1
PDHG_XT_BATCH=1 PDHG_XT_RPRE=2 run b0_rpre2 || exit 1
PDHG_XT_BATCH=1 PDHG_DBG=1 run b0_dbg1 || exit 1
PDHG_XT_BATCH=1 PDHG_DBG=2 run b0_dbg2 || exit 1
PDHG_XT_BATCH=1 PDHG_DBG=3 run b0_dbg3 || exit 1
PDHG_XT_BATCH=1 PDHG_DBG=7 run b0_dbg7 || exit 1
PDHG_XT_BATCH=0 run ws2 || exit 1
echo all-done
