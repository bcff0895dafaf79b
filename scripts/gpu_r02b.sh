# round 2: diagnose the x transform and the fused residual (SQ counters + timing with parts switched off)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02b
for D in 0 1 4 5; do
  echo "== PDHG_DBG=$D"
  PDHG_DBG=$D timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-pmc --no-cpu-baseline --no-probe > gpurun_out/r02b/dbg$D.json 2>/dev/null || exit 1
done
cd /tmp && export TMPDIR=/tmp
ARGS="$GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pmc --no-probe"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r02b/sq1 -o run -- python3 $ARGS > $GRAFT_REPO_ROOT/gpurun_out/r02b/sq1.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r02b/sq2 -o run -- python3 $ARGS > $GRAFT_REPO_ROOT/gpurun_out/r02b/sq2.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r02b/g1 -o run -- python3 $ARGS > $GRAFT_REPO_ROOT/gpurun_out/r02b/g1.log 2>&1 || exit 1
echo done
