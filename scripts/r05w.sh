#!/bin/bash
# round 5: task-order residual spectrum (fp64 C3) -- tests (bitwise vs blocked, slabs, full-size C3 fp64), A/B
set -o pipefail
mkdir -p gpurun_out/r05w
export PYTHONPATH=$PWD/pdhg-optimal-control_amd:$PWD/oracle:$PWD/tests
#timeout -k 10 800 python -u -m pytest tests/test_gpu_xt64.py tests/test_gpu_slab64.py tests/test_gpu_fullsize.py \
  tests/test_gpu_decomp.py -x -v --timeout 400 --timeout-method thread \
#  -k "task_order or 4096x4096 or c3-fp64 or (c3_p8 and fp64) or fp64_x_kernel" > gpurun_out/r05w/tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/r05w/tests.log | head; tail -5 gpurun_out/r05w/tests.log; exit 1; }
grep -E "PASSED|passed" gpurun_out/r05w/tests.log | tail -12
cp -f gpurun_out/parity.jsonl gpurun_out/r05w/parity.jsonl
AB_PREC=fp64 timeout -k 10 500 python -u scripts/ab_env.py c3 3 4 "" "PDHG_TC_SPEC=0" > gpurun_out/r05w/ab.txt 2>&1 || { tail -10 gpurun_out/r05w/ab.txt; exit 1; }
grep MEDIAN gpurun_out/r05w/ab.txt
