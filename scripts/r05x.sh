#!/bin/bash
# round 5: task-order spectrum with XCD-ordered x-kernel blocks -- bitwise test, then interleaved A/B at C3 fp64
set -o pipefail
mkdir -p gpurun_out/r05x
export PYTHONPATH=$PWD/pdhg-optimal-control_amd:$PWD/oracle:$PWD/tests
timeout -k 10 400 python -u -m pytest tests/test_gpu_xt64.py -x -v --timeout 300 --timeout-method thread -k "task_order" \
  > gpurun_out/r05x/tests.log 2>&1 || { grep -E "FAILED|assert" gpurun_out/r05x/tests.log | head; exit 1; }
grep -E "passed" gpurun_out/r05x/tests.log
AB_PREC=fp64 timeout -k 10 500 python -u scripts/ab_env.py c3 3 4 "" "PDHG_TC_SPEC=0" > gpurun_out/r05x/ab.txt 2>&1 || { tail -10 gpurun_out/r05x/ab.txt; exit 1; }
grep MEDIAN gpurun_out/r05x/ab.txt
