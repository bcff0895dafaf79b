#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per access width (scripts/fetch_calib.hip, built in-tree on the CPU side).
# usage (GPU box): bash scripts/fetch_calib.sh <tag>  -> gpurun_out/calib_<tag>/
set -o pipefail
TAG=${1:-calib}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/calib_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o run -- "$REPO/scripts/fetch_calib" > "$OUT/pmc_$C.log" 2>&1 || exit 1
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    acc = collections.defaultdict(list)
    for f in glob.glob(out + "/pmc_%s/**/*counter_collection.csv" % c, recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == c:
                acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items()):
        # FETCH_SIZE / WRITE_SIZE are in KiB; the kernels move 1 GiB each
        print("%-10s %-60s %s  ratio to 1 GiB: %s" % (c, k[:60], v, [round(x * 1024 / 2**30, 3) for x in v]))
PY
