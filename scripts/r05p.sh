#!/bin/bash
# round 5: the whole GPU suite (parity log -> gpurun_out/r05p/parity.jsonl), then smoke()
set -o pipefail
mkdir -p gpurun_out/r05p
rm -f gpurun_out/parity.jsonl
export PYTHONPATH=$PWD/pdhg-optimal-control_amd:$PWD/oracle:$PWD/tests
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/r05p/suite.log 2>&1; rc=$?
cp -f gpurun_out/parity.jsonl gpurun_out/r05p/parity.jsonl 2>/dev/null
grep -E "FAILED|ERROR" gpurun_out/r05p/suite.log | head -20
tail -3 gpurun_out/r05p/suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05p/smoke.log 2>&1; rc=$?
tail -3 gpurun_out/r05p/smoke.log
exit $rc
