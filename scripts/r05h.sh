#!/bin/bash
# round 5: fp64 x-slab decomposition tests
set -o pipefail
mkdir -p gpurun_out/r05h
export PYTHONPATH=$PWD/pdhg-optimal-control_amd:$PWD/oracle:$PWD/tests
timeout -k 10 900 python -u -m pytest tests/test_gpu_xslab.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r05h/xslab.log 2>&1
rc=$?
tail -5 gpurun_out/r05h/xslab.log
cp -f gpurun_out/parity.jsonl gpurun_out/r05h/parity.jsonl 2>/dev/null
exit $rc
