"""Summarise a scripts/profile.sh output dir: per-kernel avg duration and per-dispatch HBM bytes.

FETCH_SIZE is doubled per MI355X_MICROARCH.md §HBM (gfx950 reports half the bytes of a wide
coalesced read); both counters are in KiB."""
import csv
import collections
import os
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name).replace("void pdhg::", "")
    for k in ("k_res_fwdy_fused_2d", "k_res_fwdy_fast_2d", "k_invy_update_fast_2d", "k_precond_xt_batch_2d",
              "k_precond_xt_ws_2d", "k_precond_xt_fast_2d", "k_precond_x_t1_2d", "k_dual_lds_2d", "k_dual_fast_2d",
              "k_res_fwdy_2d", "k_precond_xt_2d", "k_invy_update_2d", "k_dual_2d", "k_res_fwdx_1d",
              "k_thomas_chunk_1d", "k_thomas_1d", "k_fs1_1d<0", "k_fs1_1d<1", "k_fs2_1d<0", "k_fs2_1d<1",
              "k_f16a_fwd_1d", "k_f16b_fwd_1d", "k_f16b_inv_1d", "k_f16a_inv_1d", "k_precond_xt_dma_2d",
              "k_fold_partials", "k_fs1w_1d<0", "k_fs1w_1d<1", "k_fs2w_1d<0", "k_fs2w_1d<1",
              "k_invx_update_1d", "k_dual_1d", "k_precond_xt_f64_2d", "k_finalize_primal", "k_finalize_dual", "k_finalize_outer",
              "k_outer_sums", "k_bcast_rows", "k_fill"):
        if k in name:
            return k
    return name[:40]


def main(d):
    dur = collections.defaultdict(list)
    with open(os.path.join(d, "trace", "run_kernel_trace.csv")) as f:
        for r in csv.DictReader(f):
            dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for sub in os.listdir(d):
        p = os.path.join(d, sub, "run_counter_collection.csv")
        if sub.startswith("pmc_") and os.path.exists(p):
            with open(p) as f:
                for r in csv.DictReader(f):
                    pmc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("{:22s} {:>6s} {:>10s} {:>12s} {:>12s} {:>9s}".format("kernel", "n", "avg_ms", "fetch_GB*2", "write_GB",
                                                                  "L2hit%"))
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        c = pmc.get(k, {})
        f = c.get("FETCH_SIZE", [])
        w = c.get("WRITE_SIZE", [])
        h, m = c.get("TCC_HIT_sum", []), c.get("TCC_MISS_sum", [])
        fs = "{:.2f}".format(2 * sum(f) / len(f) * 1024 / 1e9) if f else "-"
        ws = "{:.2f}".format(sum(w) / len(w) * 1024 / 1e9) if w else "-"
        hr = "{:.1f}".format(100 * sum(h) / (sum(h) + sum(m))) if h and (sum(h) + sum(m)) > 0 else "-"
        print("{:22s} {:6d} {:10.3f} {:>12s} {:>12s} {:>9s}".format(k, len(v), sum(v) / len(v), fs, ws, hr))


if __name__ == "__main__":
    main(sys.argv[1])
