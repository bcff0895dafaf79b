#!/bin/bash
# round 5: stream-ordered uploads / multi buffer zeroing -- the poison repro of the multi-context fp64 mismatch, then
# the fp64 decomposition tests
set -o pipefail
mkdir -p gpurun_out/r05m
export PYTHONPATH=$PWD/pdhg-optimal-control_amd:$PWD/oracle:$PWD/tests
timeout -k 10 600 python -u scripts/diag_poison.py > gpurun_out/r05m/poison.log 2>&1 || { tail -20 gpurun_out/r05m/poison.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05m/poison.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_decomp.py -v --timeout 300 --timeout-method thread -k "fp64" \
  > gpurun_out/r05m/decomp.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r05m/decomp.log | tail -12
exit $rc
