#!/bin/bash
# round 5: the tail of the GPU suite (files from test_gpu_slab64 on) with per-test durations, then smoke()
set -o pipefail
mkdir -p gpurun_out/r05q
rm -f gpurun_out/parity.jsonl
export PYTHONPATH=$PWD/pdhg-optimal-control_amd:$PWD/oracle:$PWD/tests
timeout -k 10 900 python -u -m pytest tests/test_gpu_slab64.py tests/test_gpu_xslab.py tests/test_gpu_xt64.py -m gpu -v \
  --timeout 300 --timeout-method thread --durations=15 > gpurun_out/r05q/suite.log 2>&1; rc=$?
cp -f gpurun_out/parity.jsonl gpurun_out/r05q/parity.jsonl 2>/dev/null
grep -E "FAILED|ERROR" gpurun_out/r05q/suite.log | head -20
tail -20 gpurun_out/r05q/suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05q/smoke.log 2>&1; rc=$?
tail -3 gpurun_out/r05q/smoke.log
exit $rc
