#!/bin/bash
# Extra PMC passes (one rocprofv3 run per counter group) for one bench config.
# usage: scripts/counters.sh <config> <tag> "<group1>" ["<group2>" ...]  -> gpurun_out/cnt_<tag>/
# Summarise with: python scripts/counter_summary.py gpurun_out/cnt_<tag>
set -o pipefail
CFG=$1; TAG=$2; shift 2
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/cnt_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="$REPO/bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline --no-pmc --no-probe --no-reference-precision"
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_available.txt" 2>&1 || true
i=0
for C in "$@"; do
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d "$OUT/g$i" -o run -- python3 $ARGS > "$OUT/g$i.log" 2>&1 || exit 1
  i=$((i+1))
done
echo "counters done: $OUT"
