#!/bin/bash
# rocprofv3 kernel statistics of the marching time-to-solution run (bench.py --marching; GPU box via gpurun).
# usage: scripts/prof_marching.sh <tag> [NAME=value ...] [bench args]   -> gpurun_out/prof_<tag>/
set -o pipefail
TAG=${1:-march}; shift
# leading NAME=value arguments: exported for the profiled run (A/B of tuning switches)
while [ $# -gt 0 ] && [[ $1 =~ ^[A-Z_][A-Z0-9_]*= ]]; do export "$1"; shift; done
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$REPO/bench.py" --config c2 --marching --rho-alp-iters 10 --no-cpu-baseline "$@" > "$OUT/trace.log" 2>&1 || exit 1
echo "profile done: $OUT"
