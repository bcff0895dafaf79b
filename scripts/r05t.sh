#!/bin/bash
# round 5: fp64 2-row update at ny = 8192 -- tests (fast vs generic, fused C4 plane, full-size c4w50 fp64), A/B
set -o pipefail
mkdir -p gpurun_out/r05t
export PYTHONPATH=$PWD/pdhg-optimal-control_amd:$PWD/oracle:$PWD/tests
timeout -k 10 700 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_fullsize.py -x -v --timeout 400 \
  --timeout-method thread -k "c4_plane or c4w50-fp64" > gpurun_out/r05t/tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/r05t/tests.log | head; tail -5 gpurun_out/r05t/tests.log; exit 1; }
grep -E "PASSED|passed" gpurun_out/r05t/tests.log | tail -6
AB_PREC=fp64 timeout -k 10 400 python -u scripts/ab_env.py c4w50 2 4 "" "PDHG_UPD8192=0" > gpurun_out/r05t/ab.txt 2>&1 || { tail -10 gpurun_out/r05t/ab.txt; exit 1; }
grep MEDIAN gpurun_out/r05t/ab.txt
