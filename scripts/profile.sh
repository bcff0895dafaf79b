#!/bin/bash
# rocprofv3 kernel trace + PMC passes for one bench config (run on the GPU box via gpurun).
# usage: scripts/profile.sh <config> <tag> [extra bench args, e.g. --precision fp64]   -> gpurun_out/prof_<tag>/...
set -o pipefail
CFG=${1:-c3}; TAG=${2:-$CFG}; shift 2; EXTRA="$*"
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
# the bench's own step counts (10 timed after 3 warm-up), so the trace's per-kernel averages are those of its line
ARGS="$REPO/bench.py --config $CFG --steps 10 --warmup 3 --no-cpu-baseline --no-pmc --no-probe --no-reference-precision $EXTRA"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $ARGS > "$OUT/trace.log" 2>&1 || exit 1
[ "${PROF_PMC:-1}" = 0 ] && { echo "profile done (trace only): $OUT"; exit 0; }   # PROF_PMC=0: kernel trace only
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  N=$(echo $C | tr ' ' '_')
  timeout -k 10 400 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$N" -o run -- python3 $ARGS > "$OUT/pmc_$N.log" 2>&1 || exit 1
done
echo "profile done: $OUT"
