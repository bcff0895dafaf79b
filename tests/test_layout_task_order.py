"""CPU check of the task-order residual spectrum's index math (fp64 C3, PDHG_TC_SPEC): the offset at which the
residual kernels store the value of row x, column ky (k_res_fwdy_fast_2d / k_res_fwdy_fused_2d: run per 4-row task,
float4 number t = b * CS4 + part of unpack_chunk4, element e = rows 2 part + e / 2, column 2 b + e % 2) equals the
offset the x kernel's forward sweep loads item (x, ky) from (k_precond_xt_f64_2d<..., TC>: block b = ky / 2, lane
tid = x % NT, item i = x / NT, byte offset 64 b + 32 ny (tid / 4) + 16 (tid % 4) + 8 ny NT i, plus 8 for ky odd),
and every value has its own slot (the run of a task is exactly the region of its R rows)."""
import numpy as np


def store_offset(x, ky, ny, rw=4, B=2):
    x0, r = (x // rw) * rw, x % rw
    b, c = ky // B, ky % B
    cs4 = rw * B // 4
    part, e = r // 2, 2 * (r % 2) + c          # unpack_chunk4 (B = 2): (a0, a1, b0, b1) = rows 2p, 2p+1 x columns
    t = b * cs4 + part
    return x0 * ny + 4 * t + e                 # reals from the row's base


def load_offset(x, ky, ny, NT=512):
    b, c = ky // 2, ky % 2
    tid, i = x % NT, x // NT
    byte = 64 * b + 32 * ny * (tid >> 2) + 16 * (tid & 3) + 8 * ny * NT * i + 8 * c
    return byte // 8


def test_task_order_offsets_agree():
    nx = ny = 4096
    rng = np.random.default_rng(0)
    xs = np.concatenate([np.arange(16), rng.integers(0, nx, 400), [nx - 1]])
    kys = np.concatenate([np.arange(16), rng.integers(0, ny, 400), [ny - 1]])
    for x in xs:
        for ky in kys[:64]:
            assert store_offset(int(x), int(ky), ny) == load_offset(int(x), int(ky), ny), (x, ky)
    # a small grid: a bijection onto the row, each task's run = the region of its own rows
    nxs, nys = 16, 8
    offs = {store_offset(x, ky, nys) for x in range(nxs) for ky in range(nys)}
    assert offs == set(range(nxs * nys))
    for x in range(nxs):
        lo = (x // 4) * 4 * nys
        assert all(lo <= store_offset(x, ky, nys) < lo + 4 * nys for ky in range(nys))
