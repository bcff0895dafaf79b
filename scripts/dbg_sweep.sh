#!/bin/bash
# Timing experiments: the C3 bench line with parts of the kernels switched off through PDHG_DBG (the results are
# numerically wrong; only the per-class kernel times are of interest).  Bits: 1 x-transform forward FFT off,
# 2 x-transform inverse FFT off, 16 fused-residual FFT off, 32 fused-residual unpack/stores off, 64 update FFT off,
# 128 dual rho / alp stores off, 256 dual residual / edge terms off.
# usage: scripts/dbg_sweep.sh <config> <dbg values...>   -> one JSON line per value with the class times
set -o pipefail
CFG=$1; shift
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO"
for D in "$@"; do
  PDHG_DBG=$D timeout -k 10 300 python bench.py --config "$CFG" --steps 6 --warmup 2 --no-pmc --no-cpu-baseline --no-probe --no-reference-precision \
    2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'dbg': $D, 'ms_per_step': round(d['ms_per_step'],2), 'kernels': {k: round(v['avg_ms'],3) for k, v in d['kernels'].items()}}))" || exit 1
done
