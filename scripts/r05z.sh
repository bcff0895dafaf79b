#!/bin/bash
# round 5 final: the GPU suite in two halves (this script: half $1 = a | b), parity log per half, smoke() after b
set -o pipefail
H=${1:-a}
mkdir -p gpurun_out/r05z
rm -f gpurun_out/parity.jsonl
export PYTHONPATH=$PWD/pdhg-optimal-control_amd:$PWD/oracle:$PWD/tests
if [ "$H" = a ]; then
  FILES="tests/test_golden.py tests/test_run_example.py tests/test_gpu_configs.py tests/test_gpu_decomp.py tests/test_gpu_divergence.py tests/test_gpu_dual_multi.py tests/test_gpu_fullsize.py"
else
  FILES="tests/test_gpu_fused.py tests/test_gpu_multi.py tests/test_gpu_parity.py tests/test_gpu_res64.py tests/test_gpu_slab.py tests/test_gpu_slab64.py tests/test_gpu_xslab.py tests/test_gpu_xt64.py"
fi
timeout -k 10 1100 python -u -m pytest $FILES -m gpu -v --timeout 400 --timeout-method thread --durations=10 \
  > gpurun_out/r05z/suite_$H.log 2>&1; rc=$?
cp -f gpurun_out/parity.jsonl gpurun_out/r05z/parity_$H.jsonl 2>/dev/null
grep -E "FAILED|ERROR" gpurun_out/r05z/suite_$H.log | head -20
tail -14 gpurun_out/r05z/suite_$H.log
[ $rc -eq 0 ] || exit $rc
if [ "$H" = b ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05z/smoke.log 2>&1; rc=$?
  tail -2 gpurun_out/r05z/smoke.log
fi
exit $rc
