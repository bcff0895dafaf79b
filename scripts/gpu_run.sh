#!/bin/bash
# One parameterised GPU-box script (replaces the per-experiment gpu_r02*.sh files).
# usage (via gpurun): bash scripts/gpu_run.sh <tag> <step> [<step> ...]
#   info                  rocm-smi clocks / power / product (which box a timing came from)
#   smoke                 __graft_entry__.smoke()
#   tests[:<pytest -k>]   pytest -m gpu (optionally filtered)
#   bench[:<args>]        python bench.py <args, commas for spaces>  -> bench_<n>.json
#                         (leading NAME=value arguments of bench / py / prof / sh steps go to that step's environment)
#   prof:<config>[,args]  scripts/profile.sh <config> <tag> [bench args]
#   sh:<script>,<args>    bash <script> <args> ('+' inside an argument stands for a space: counter groups)
# Every GPU step runs under its own time limit; the first failure ends the script.
set -o pipefail
TAG=$1; shift
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
  arg=${arg//,/ }
  # leading NAME=value tokens of a bench / py step are set in that step's environment only
  ENVV=()
  if [ "$kind" = bench ] || [ "$kind" = py ] || [ "$kind" = prof ] || [ "$kind" = sh ]; then
    read -ra TOK <<< "$arg"
    while [ ${#TOK[@]} -gt 0 ] && [[ ${TOK[0]} =~ ^[A-Z_][A-Z0-9_]*= ]]; do ENVV+=("${TOK[0]}"); TOK=("${TOK[@]:1}"); done
    arg="${TOK[*]}"
  fi
  echo "[$(date +%T)] step $n: $kind ${ENVV[*]} $arg"
  case $kind in
    info)  { timeout -k 5 60 rocm-smi --showproductname --showclocks --showpower --showtemp --showperflevel; hostname; } > "$OUT/info_$n.log" 2>&1
           grep -E "sclk|mclk|Power|Perf|Card SKU" "$OUT/info_$n.log" | head -12 || true ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed rc=$?"; tail -20 "$OUT/smoke.log"; exit 1; } ;;
    tests) arg=${arg//+/ }; if [ -n "$arg" ]; then K=(-k "$arg"); else K=(); fi
           timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread "${K[@]}" > "$OUT/tests_$n.log" 2>&1 || { echo "tests failed rc=$?"; tail -30 "$OUT/tests_$n.log"; exit 1; }
           tail -3 "$OUT/tests_$n.log" ;;
    bench) env "${ENVV[@]}" timeout -k 10 900 python -u bench.py $arg > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" || { echo "bench failed rc=$?"; tail -20 "$OUT/bench_$n.err"; exit 1; }
           cat "$OUT/bench_$n.json" ;;
    prof)  read -ra TOK <<< "$arg"; PT="${TAG}_$(echo "${TOK[*]}" | tr -c 'A-Za-z0-9_\n' '_')"
           env "${ENVV[@]}" timeout -k 10 1000 bash scripts/profile.sh "${TOK[0]}" "$PT" "${TOK[@]:1}" > "$OUT/prof_$n.log" 2>&1 || { echo "prof failed rc=$?"; tail -20 "$OUT/prof_$n.log"; exit 1; }
           echo "profile: gpurun_out/prof_$PT"
           cd "$REPO" ;;
    py)    env "${ENVV[@]}" timeout -k 10 900 python -u $arg > "$OUT/py_$n.log" 2>&1 || { echo "py failed rc=$?"; tail -30 "$OUT/py_$n.log"; exit 1; }
           tail -40 "$OUT/py_$n.log" ;;
    sh)    read -ra TOK <<< "$arg"; TOK=("${TOK[@]//+/ }")
           env "${ENVV[@]}" timeout -k 10 1100 bash "${TOK[@]}" > "$OUT/sh_$n.log" 2>&1 || { echo "sh failed rc=$?"; tail -20 "$OUT/sh_$n.log"; exit 1; }
           tail -5 "$OUT/sh_$n.log"; cd "$REPO" ;;
    *) echo "unknown step $kind"; exit 2 ;;
  esac
done
echo all-done
