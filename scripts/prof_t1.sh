#!/bin/bash
# rocprofv3 kernel trace of the T = 1 steady-state iteration (scripts/diag_t1_iter.py) for one variant.
# usage (via gpurun / gpu_run.sh sh:): bash scripts/prof_t1.sh <tag> <iters> "<VAR=value ...>"
set -o pipefail
TAG=$1; IT=${2:-2000}; VAR=${3:-PDHG_SPEC=1}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/prof_t1_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$REPO/scripts/diag_t1_iter.py" "$IT" 1 "$VAR" > "$OUT/trace.log" 2>&1 || exit 1
echo "profile done: $OUT"
