#!/bin/bash
# round 5: fp64 x-slab marching test + c3w1 x-slab bench records (fp64 / fp32) and the single-context fp64 line
set -o pipefail
mkdir -p gpurun_out/r05i
export PYTHONPATH=$PWD/pdhg-optimal-control_amd:$PWD/oracle:$PWD/tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_xslab.py -x -v --timeout 300 --timeout-method thread \
  -k "multi_step" > gpurun_out/r05i/tests.log 2>&1 || { tail -30 gpurun_out/r05i/tests.log; exit 1; }
tail -4 gpurun_out/r05i/tests.log
B="--steps 50 --warmup 5 --no-cpu-baseline --no-pmc --no-probe --no-reference-precision"
timeout -k 10 300 python -u bench.py --config c3w1 --decomp xslab --precision fp64 $B > gpurun_out/r05i/xslab64.json 2> gpurun_out/r05i/xslab64.err && \
timeout -k 10 300 python -u bench.py --config c3w1 --decomp xslab --precision fp32 $B > gpurun_out/r05i/xslab32.json 2> gpurun_out/r05i/xslab32.err && \
timeout -k 10 300 python -u bench.py --config c3w1 --precision fp64 $B > gpurun_out/r05i/single64.json 2> gpurun_out/r05i/single64.err
rc=$?
for f in xslab64 xslab32 single64; do python -c "import json,sys; d=json.load(open('gpurun_out/r05i/$f.json')); print('$f', d['value'], d['ms_per_step'], d.get('kernels_ms'))" ; done
exit $rc
