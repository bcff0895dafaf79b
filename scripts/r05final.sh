#!/bin/bash
# round 5: the default bench line (fp64 C3 headline + nested fp32, PMC passes, CPU baseline) and a rocprofv3
# kernel-trace summary of the same command
set -o pipefail
mkdir -p gpurun_out/r05final
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py > gpurun_out/r05final/bench_default.json 2> gpurun_out/r05final/bench_default.err || { tail -20 gpurun_out/r05final/bench_default.err; exit 1; }
cat gpurun_out/r05final/bench_default.json | head -c 400; echo
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r05final/prof -o run -- python3 bench.py --steps 10 --warmup 3 \
  --no-cpu-baseline --no-pmc --no-probe --no-reference-precision > gpurun_out/r05final/prof.json 2> gpurun_out/r05final/prof.err || { tail -20 gpurun_out/r05final/prof.err; exit 1; }
find gpurun_out/r05final/prof -name "*stats*"
