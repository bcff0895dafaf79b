#!/bin/bash
# usage: scripts/sweep_env.sh VAR "v1 v2 ..." [bench args]  -> one bench line per value (no PMC / CPU leg)
VAR=$1; VALS=$2; shift 2
for v in $VALS; do
  echo "== $VAR=$v"
  env $VAR=$v timeout -k 10 300 python bench.py --no-pmc --no-cpu-baseline --no-reference-precision "$@" | python -c "
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1])
print('it/s %.3f' % d['value'], {k: round(v['avg_ms'],2) for k,v in d['kernels'].items()})" || exit 1
done
