"""Per-kernel VGPR / AGPR / scratch / occupancy of libpdhg's device code, from the compiler's
kernel-resource-usage remarks (static check, CPU only).
usage: python scripts/resource_usage.py [substring ...]   (compiles pdhg_api.hip device-only, ~2 min;
       PDHG_RU_LOG=<file> reuses a saved remark log)"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "pdhg-optimal-control_amd", "csrc", "pdhg_api.hip")


def remarks():
    log = os.environ.get("PDHG_RU_LOG")
    if log and os.path.exists(log):
        return open(log).read()
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-value",
           "-Wno-unused-result", "--cuda-device-only", "-c", "-o", "/tmp/pdhg_ru.o", SRC,
           "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if log:
        open(log, "w").write(r.stderr)
    return r.stderr


def parse(txt):
    rows, cur = {}, None
    for ln in txt.splitlines():
        if "kernel-resource-usage" not in ln:
            continue
        m = re.search(r"remark:\s+(.*?): (\S+) \[-Rpass", ln)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2)
        if k == "Function Name":
            cur = v
            rows[cur] = {}
        elif cur:
            rows[cur][k] = v
    return rows


def main():
    rows = parse(remarks())
    names = list(rows)
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
    pats = sys.argv[1:]
    for n, d in zip(names, dem):
        if pats and not any(p in d for p in pats):
            continue
        r = rows[n]
        print("{:<110} vgpr {:>3} agpr {:>3} scratch {:>4} occ {:>2} lds {:>6}".format(
            d[:110], r.get("VGPRs"), r.get("AGPRs"), r.get("ScratchSize [bytes/lane]"),
            r.get("Occupancy [waves/SIMD]"), r.get("LDS Size [bytes/block]")))


if __name__ == "__main__":
    main()
