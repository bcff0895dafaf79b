"""Static check of the LDS-DMA x transform's counted wait (CPU, no GPU needed).

k_precond_xt_dma_2d (csrc/kernels_xt_dma.hpp) stages the next batch's rows HBM -> LDS with global_load_lds and
retires them one batch later with a counted ``s_waitcnt vmcnt(4)``: the 4 stores of a full batch are the only
vector-memory ops issued after the DMA, so waiting until at most 4 are outstanding means the (older) DMA has
landed.  The staged rows are then read by inline-asm ds_reads the compiler cannot see as depending on the DMA,
so the wait is only correct if the generated code really issues >= N vector-memory ops between the last DMA
and every ``vmcnt(N)`` (N > 0).  This test disassembles the built library and checks exactly that, in program
order, for every counted wait of the kernel -- a compiler schedule that moved a store above the DMA (or dropped
one) fails here instead of reading unlanded rows on the GPU.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "pdhg-optimal-control_amd", "pdhg_amd", "libpdhg.so")
LLVM = "/opt/rocm/lib/llvm/bin"
TOOLS = [os.path.join(LLVM, t) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump")]
VMEM = re.compile(r"^\s*(global_|buffer_|flat_|scratch_)")


def _disassemble(tmp_path):
    fb, co = tmp_path / "fatbin.bin", tmp_path / "gfx950.o"
    subprocess.run([TOOLS[0], "--dump-section", ".hip_fatbin={}".format(fb), LIB, str(tmp_path / "junk.so")],
                   check=True, capture_output=True)
    subprocess.run([TOOLS[1], "--unbundle", "--type=o", "--input={}".format(fb),
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output={}".format(co)],
                   check=True, capture_output=True)
    out = subprocess.run([TOOLS[2], "-d", "--mcpu=gfx950", str(co)], check=True, capture_output=True, text=True)
    return out.stdout.splitlines()


def _kernel_bodies(lines, name_part):
    """{symbol: body} of every kernel whose symbol contains name_part."""
    out, start, name = {}, None, None
    for i, ln in enumerate(lines + ["0 <end>:"]):
        if re.match(r"^[0-9a-f]+ <.*>:", ln):
            if start is not None:
                out[name] = lines[start:i]
                start = None
            if name_part in ln:
                start, name = i, ln
    return out


@pytest.mark.skipif(not os.path.exists(LIB), reason="libpdhg.so not built (run __graft_entry__.build())")
@pytest.mark.skipif(not all(os.path.exists(t) or shutil.which(os.path.basename(t)) for t in TOOLS),
                    reason="ROCm LLVM tools absent")
def test_dma_counted_waits_cover_the_dma(tmp_path):
    """Both instantiations: k_precond_xt_dma_2d<4096> (column pairs) and <4096, true> (half-real, C4's nx = 8192,
    whose backward batch stores 8 float2 instead of 4 float4 -- the vmcnt(4) then over-waits, still safe)."""
    bodies = _kernel_bodies(_disassemble(tmp_path), "k_precond_xt_dma_2dILi4096E")
    assert len(bodies) == 2, "expected k_precond_xt_dma_2d<4096, false / true> in libpdhg.so: {}".format(list(bodies))
    for body in bodies.values():
        _check(body)


def _check(body):
    counted = 0
    for i, ln in enumerate(body):
        m = re.search(r"s_waitcnt\s+vmcnt\((\d+)\)", ln)
        if not m or int(m.group(1)) == 0:
            continue
        need = int(m.group(1))
        after = 0   # vector-memory ops between the nearest preceding DMA and this wait
        dma_seen = False
        for prev in reversed(body[:i]):
            if "global_load_lds" in prev:
                dma_seen = True
                break
            if VMEM.match(prev.split("//")[0]):
                after += 1
        assert dma_seen, "a counted wait with no DMA before it: line {}".format(ln.strip())
        assert after >= need, ("vmcnt({}) with only {} vector-memory ops after the last DMA: the staged rows "
                               "could be read before they land ({})".format(need, after, ln.strip()))
        counted += 1
    # the kernel's schedule this test pins: one counted wait per copy of the batch loop
    assert counted >= 1, "no counted vmcnt wait left in k_precond_xt_dma_2d (schedule changed: re-check it)"
