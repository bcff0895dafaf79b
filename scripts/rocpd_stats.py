"""Kernel statistics (the rocprofv3 --stats summary: calls, total / average / min / max duration, share) from a
rocprofv3 SQLite output (<dir>/<name>_results.db), with each kernel's VGPR / AGPR / scratch / LDS from its dispatches.
usage: python scripts/rocpd_stats.py <results.db> [out.csv]"""
import csv
import sqlite3
import sys


def main():
    db, out = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else None)
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
                     "max(vgpr_count), max(accum_vgpr_count), max(scratch_size), max(lds_size) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    hdr = ["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage", "VGPR", "AGPR",
           "ScratchBytes", "LdsBytes"]
    table = [[r[0], r[1], int(r[2]), round(r[3], 1), int(r[4]), int(r[5]), round(100.0 * r[2] / total, 2)] +
             list(r[6:]) for r in rows]
    w = csv.writer(open(out, "w", newline="") if out else sys.stdout)
    w.writerow(hdr)
    w.writerows(table)


if __name__ == "__main__":
    main()
