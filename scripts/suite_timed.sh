#!/bin/bash
# GPU suite (or a part of it) with per-test durations: junit xml + --durations=0 under gpurun_out/<tag>/.
# usage (via gpurun): bash scripts/suite_timed.sh <tag> <limit_s> [pytest args: files / -k ...]
set -o pipefail
TAG=$1; LIM=$2; shift 2
mkdir -p gpurun_out/$TAG
rm -f gpurun_out/parity.jsonl
timeout -k 10 "$LIM" python -u -m pytest "$@" -m gpu -q -x --timeout 300 --timeout-method thread \
  --durations=0 --junitxml=gpurun_out/$TAG/junit.xml > gpurun_out/$TAG/suite.log 2>&1; rc=$?
cp -f gpurun_out/parity.jsonl gpurun_out/$TAG/parity.jsonl 2>/dev/null
grep -E "FAILED|ERROR|passed|failed" gpurun_out/$TAG/suite.log | tail -20
exit $rc
