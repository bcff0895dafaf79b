"""Per-file and slowest-test durations of a GPU suite run from its junit xml (scripts/suite_timed.sh writes it).

usage: python scripts/junit_durations.py gpurun_out/<tag>/junit.xml [top_n] > profiles/<name>.txt"""
import collections
import sys
import xml.etree.ElementTree as ET


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    rows, skipped = [], 0
    for tc in ET.parse(path).iter("testcase"):
        if tc.find("skipped") is not None:
            skipped += 1
            continue
        rows.append((float(tc.get("time")), "{}::{}".format(tc.get("classname"), tc.get("name"))))
    total = sum(t for t, _ in rows)
    print("# {}: {} tests run, {} skipped, {:.1f} s of test time".format(path, len(rows), skipped, total))
    agg = collections.defaultdict(lambda: [0.0, 0])
    for t, n in rows:
        a = agg[n.split("::")[0]]
        a[0] += t
        a[1] += 1
    print("\n# per file: seconds, tests")
    for f, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        print("{:8.1f} {:4d}  {}".format(t, c, f))
    print("\n# slowest {} tests (the first test of the run carries the process's import / HIP start-up)".format(top))
    for t, n in sorted(rows, reverse=True)[:top]:
        print("{:8.1f}  {}".format(t, n))


if __name__ == "__main__":
    main()
