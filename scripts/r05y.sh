#!/bin/bash
# round 5: task-order spectrum in the fused residual's R plane -- tests (bitwise vs blocked, slabs, full-size C3
# fp64, decomposition), then A/B incl. the x kernel's XCD order (PDHG_DBG=4096: round robin)
set -o pipefail
mkdir -p gpurun_out/r05y
export PYTHONPATH=$PWD/pdhg-optimal-control_amd:$PWD/oracle:$PWD/tests
timeout -k 10 800 python -u -m pytest tests/test_gpu_xt64.py tests/test_gpu_slab64.py tests/test_gpu_fullsize.py \
  tests/test_gpu_decomp.py tests/test_gpu_fused.py -x -v --timeout 400 --timeout-method thread \
  -k "task_order or 4096x4096 or c3-fp64 or (c3_p8 and fp64) or fused_fp64" > gpurun_out/r05y/tests.log 2>&1 || { grep -E "FAILED|assert" gpurun_out/r05y/tests.log | head; tail -3 gpurun_out/r05y/tests.log; exit 1; }
grep -E "passed" gpurun_out/r05y/tests.log
cp -f gpurun_out/parity.jsonl gpurun_out/r05y/parity.jsonl
AB_PREC=fp64 timeout -k 10 600 python -u scripts/ab_env.py c3 3 4 "" "PDHG_DBG=4096" "PDHG_TC_SPEC=0" > gpurun_out/r05y/ab.txt 2>&1 || { tail -10 gpurun_out/r05y/ab.txt; exit 1; }
grep MEDIAN gpurun_out/r05y/ab.txt
