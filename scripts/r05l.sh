#!/bin/bash
# round 5: XCD-aware task order of the fused residual -- interleaved A/B (PDHG_DBG=1024 = round-robin order)
set -o pipefail
mkdir -p gpurun_out/r05l
AB_PREC=fp64 timeout -k 10 500 python -u scripts/ab_env.py c4w50 2 4 "" "PDHG_DBG=1024" > gpurun_out/r05l/c4w50_fp64.txt 2>&1 || { tail -20 gpurun_out/r05l/c4w50_fp64.txt; exit 1; }
tail -12 gpurun_out/r05l/c4w50_fp64.txt
AB_PREC=fp64 timeout -k 10 400 python -u scripts/ab_env.py c3 3 5 "" "PDHG_DBG=1024" > gpurun_out/r05l/c3_fp64.txt 2>&1 || { tail -20 gpurun_out/r05l/c3_fp64.txt; exit 1; }
tail -12 gpurun_out/r05l/c3_fp64.txt
timeout -k 10 400 python -u scripts/ab_env.py c3 3 8 "" "PDHG_DBG=1024" > gpurun_out/r05l/c3_fp32.txt 2>&1 || { tail -20 gpurun_out/r05l/c3_fp32.txt; exit 1; }
tail -12 gpurun_out/r05l/c3_fp32.txt
