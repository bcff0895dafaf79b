#!/bin/bash
# round 5: C4 16-B chunk ordering -- interleaved A/B at c4w50 fp32 (unfused: 8-group tiles vs 4 (DBG 2048);
# fused: XCD order vs round robin (DBG 1024)) and fp64
set -o pipefail
mkdir -p gpurun_out/r05n
timeout -k 10 500 python -u scripts/ab_env.py c4w50 2 4 "" "PDHG_DBG=2048" "PDHG_FUSE_RES=1" "PDHG_FUSE_RES=1 PDHG_DBG=1024" > gpurun_out/r05n/c4w50_fp32.txt 2>&1 || { tail -20 gpurun_out/r05n/c4w50_fp32.txt; exit 1; }
grep MEDIAN gpurun_out/r05n/c4w50_fp32.txt
