"""Per-kernel mean of every counter collected by scripts/counters.sh (one row per kernel class)."""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import short  # noqa: E402


def main(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in sorted(glob.glob(os.path.join(d, "g*", "run_counter_collection.csv"))):
        with open(p) as f:
            for r in csv.DictReader(f):
                acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, c in acc.items():
        if k.startswith("k_finalize") or k.startswith("k_fill") or k.startswith("k_bcast"):
            continue
        print(k)
        for n, v in sorted(c.items()):
            print("   {:28s} {:16.4g}".format(n, sum(v) / len(v)))


if __name__ == "__main__":
    main(sys.argv[1])
