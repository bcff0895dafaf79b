"""One-off (round 5): re-price the round-4 chunked-dual bench records with the bytes that crossed HBM.

bench.py of round 4 priced the chunked dual loop (kernels_dual_multi.hpp) at the per-sub-iteration bytes times the
inner count, but a pass keeps 5 sub-iterations in registers and reads / writes the state once (VERDICT r4, weak #7:
frac 2.01 / 2.34, hbm_gbps_iteration above the 8 TB/s peak).  Every listed record had inner count 10 (no early exit):
the all-chunk form runs 2 passes, the head form 1 per-sub-iteration launch + 2 chunk passes.  The measured times are
kept; roofline / hbm_gbps_iteration are recomputed from the pass bytes and the originals kept under
"as_reported_r04".  PMC dual bytes in these records are per KERNEL launch (one chunk pass), not per outer iteration."""
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RECORDS = {   # file: (passes per outer iteration, dual "launches" (ProfScopes) per outer iteration)
    "r04_bench_c2_fp64_k10_chunked_dual.json": (2, 1),
    "r04_bench_c3_k10_allchunks.json": (2, 1),
    "r04_bench_c3_k10_chunked_dual.json": (2, 1),
    "r04_bench_c3_k10_headform.json": (3, 2),
}

for name, (passes, scopes) in RECORDS.items():
    path = os.path.join(ROOT, "profiles", name)
    d = json.load(open(path))
    if "as_reported_r04" in d:
        continue
    k = 10
    dual = d["kernels"]["dual"]
    iters = d["config"]["iters_executed"]
    # one sub-iteration's algorithmic bytes (11 N S): the all-chunk records stored inner x that, the head form one
    sub = dual["bytes_per_launch"] / (k if scopes == 1 else 1)
    dual_ms_iter = dual["avg_ms"] * dual["launches"] / iters
    pass_bytes = passes * sub
    it_bytes = d["iteration_bytes"] - k * sub + pass_bytes
    d["as_reported_r04"] = {"roofline": dict(d["roofline"]), "hbm_gbps_iteration": d["hbm_gbps_iteration"],
                            "iteration_bytes": d["iteration_bytes"], "dual": dict(dual)}
    d["kernels"]["dual"] = dict(dual, bytes_per_launch=pass_bytes, avg_ms=dual_ms_iter, launches=iters,
                                passes=passes, passes_note="re-priced r05: passes x one sub-iteration's bytes")
    if "pmc_bytes_per_launch" in dual:
        d["kernels"]["dual"]["pmc_bytes_per_launch_note"] = "per kernel launch (one pass), not per outer iteration"
    ach = pass_bytes / (dual_ms_iter * 1e-3) / 1e9
    d["roofline"].update(achieved=ach, frac=ach / d["roofline"]["peak"], kernel="dual")
    d["roofline"].pop("traffic", None)
    d["roofline"]["traffic"] = None
    d["roofline"]["traffic_note"] = "round-4 PMC dual bytes were per chunk-pass launch; see as_reported_r04"
    d["iteration_bytes"] = it_bytes
    d["hbm_gbps_iteration"] = it_bytes / (d["ms_per_step"] * 1e-3) / 1e9
    d["repriced"] = "scripts/fix_r04_dual_records.py (round 5)"
    json.dump(d, open(path, "w"), indent=None)
    print(name, "frac {:.3f} hbm {:.0f} GB/s".format(d["roofline"]["frac"], d["hbm_gbps_iteration"]))
