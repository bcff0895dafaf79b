#!/bin/bash
# interleaved A/B of NAME=value switches on the marching time to solution (C2 fp64, first W windows)
# usage: scripts/ab_march.sh <rounds> <windows> "<vars A>" "<vars B>" ...   ("" = defaults); lines -> stdout
set -o pipefail
R=$1; W=$2; shift 2
for r in $(seq 1 $R); do
  for v in "$@"; do
    out=$(env $v timeout -k 10 300 python -u bench.py --config c2 --marching --rho-alp-iters 10 --windows $W \
          --no-cpu-baseline 2>/dev/null | tail -1) || exit 1
    echo "round $r [$v] $(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],3), d['total_outer_iters'])")"
  done
done
