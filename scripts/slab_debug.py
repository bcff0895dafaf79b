"""Debug helper: slab phases vs the single-context path on one GPU (prints relative differences)."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "tests"), os.path.join(os.path.dirname(__file__), "..", "oracle"),
                os.path.join(os.path.dirname(__file__), "..", "pdhg-optimal-control_amd")]
import numpy as np
import torch
from _problems import make_problem, rel
from pdhg_amd.context import PDHGContext
from pdhg_amd.slab import SlabContext, LocalComm, SlabRunner, split_state, join_state, slab_bounds

nx, ny, T = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
P = make_problem(1, 2, nx, ny, T, 0.0)
tau, sigma = 0.1 / 1.5, 0.15
ref = PDHGContext(1, 2, nx, ny, T, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"], precision="fp32")
ref.set_state(P["phi"], P["rho"], P["alp"])
ref.update_primal(tau)
phi_r = ref.get_state()[0]
for nr in (1, 2, 3):
    slabs = [SlabContext(r, nr, T, 1, nx, ny, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"]) for r in range(nr)]
    for s, part in zip(slabs, split_state(P["phi"], P["rho"], P["alp"], slab_bounds(T, nr))):
        s.set_state(*part)
    R = SlabRunner(slabs, LocalComm(nr))
    for s in slabs:
        s.begin()
    S, B, C = R.slabs, R.b, R.comm
    for s, b in zip(S, B):
        s.plane_out(0, b["rho_send"])
    C.shift_up([b["rho_send"] for b in B], [b["rho_recv"] for b in B])
    for s, b in zip(S, B):
        if not s.last:
            s.plane_in(0, b["rho_recv"])
    for s in S:
        s.forward(tau)
    for s, b in zip(S, B):
        s.plane_out(2, b["D"])
    allD = C.allgather([b["D"] for b in B])
    for i, s in enumerate(S):
        s.fixup(allD[i], R.allG[i]); s.plane_out(3, B[i]["X0"])
    allX0 = C.allgather([b["X0"] for b in B])
    for i, s in enumerate(S):
        s.backward(tau, allX0[i], R.allG[i], B[i]["sums"])
    torch.cuda.synchronize()
    phi_s = join_state([s.get_state() for s in S])[0]
    per_row = [float(rel(phi_s[j], phi_r[j])) for j in range(T + 1)]
    print("P", nr, "primal rel", rel(phi_s, phi_r), "per row", ["%.1e" % v for v in per_row])
    print("   G", [float(R.allG[0][q].abs().max()) for q in range(nr)], "D max", [float(allD[0][q].abs().max()) for q in range(nr)])
