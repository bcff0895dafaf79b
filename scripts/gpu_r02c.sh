# round 2: config parity on the available fixtures, the row-batched x transform (parity + timing)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02c
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -v -s --timeout 300 --timeout-method thread -k "c3_ws_T200 or c3_rows or c4_rows or c1_exact or one_step or batched" > gpurun_out/r02c/configs.log 2>&1; echo "configs rc=$?"
for B in 0 1; do
  PDHG_XT_BATCH=$B timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-pmc --no-cpu-baseline --no-probe > gpurun_out/r02c/bench_batch$B.json 2>gpurun_out/r02c/bench_batch$B.err || exit 1
done
PDHG_XT_BATCH=1 timeout -k 10 200 python bench.py --config c2 --steps 10 --warmup 2 --no-pmc --no-cpu-baseline --no-probe > gpurun_out/r02c/bench_c2_batch1.json 2>/dev/null || exit 1
PDHG_XT_BATCH=0 timeout -k 10 200 python bench.py --config c2 --steps 10 --warmup 2 --no-pmc --no-cpu-baseline --no-probe > gpurun_out/r02c/bench_c2_batch0.json 2>/dev/null || exit 1

for H in 2 0; do
  PDHG_HALF_NT=$H PDHG_XT_BATCH=1 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-pmc --no-cpu-baseline --no-probe > gpurun_out/r02c/bench_halfnt$H.json 2>/dev/null || exit 1
done
echo all-done2
