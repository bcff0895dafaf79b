#!/bin/bash
# A/B timing: bench.py of another tree (e.g. an older build copied under ab_*/) against this one, on one box.
# usage: scripts/ab_bench.sh <dir>[:<dir>...] [bench args]   -> one summary line per tree
set -o pipefail
DIRS=$1; shift
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
IFS=: read -ra DS <<< "$DIRS"
for d in "${DS[@]}"; do
  cd "$REPO/$d" || exit 1
  echo "== $d"
  timeout -k 10 300 python bench.py --no-pmc --no-cpu-baseline --no-probe --no-reference-precision "$@" 2>/dev/null | python -c "
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1])
print('it/s %.3f ms %.2f' % (d['value'], d['ms_per_step']), {k: round(v['avg_ms'],2) for k,v in d['kernels'].items()})" || exit 1
done
