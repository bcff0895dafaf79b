#!/bin/bash
# round 5: fp64 fused residual with 1024 threads (spills 108 B) vs 512 -- interleaved A/B at C3 fp64
set -o pipefail
mkdir -p gpurun_out/r05r
AB_PREC=fp64 timeout -k 10 500 python -u scripts/ab_env.py c3 3 5 "" "PDHG_RES64_NT=1024" > gpurun_out/r05r/c3_fp64.txt 2>&1 || { tail -20 gpurun_out/r05r/c3_fp64.txt; exit 1; }
grep MEDIAN gpurun_out/r05r/c3_fp64.txt
