"""Static guard on the streamed-weight kernels' inline-asm loads (CPU only: hipcc -S for gfx950).

The B-fragment loads of bcfft_dmk / bcfft_dm256 / bcfft_dm64k are inline-asm
`buffer_load_dwordx4` into VGPRs, waited for by hand-counted `s_waitcnt vmcnt(N)` (so the
compiler's own waits never drain the x DMA). The compiler treats an asm output as written when the
statement ends: it may copy, spill or reuse those registers before the load has landed. Round 5's
failing dmk variant (younger waves' x DMA after their stage 1, `-DBCFFT_DMK_LATE_DMA=1`: wrong
tokens at N = 4090 on the GPU, `profiles/r06_dmk_late_dma_repro.txt`) is exactly that: hipcc rotated
the 64 fragment registers with v_mov copies across the chunk loop while the loads were in flight
(DESIGN.md section 6b). The same class sat latent in the product dm256k kernel (a rotation around
stage 3 at each tile start, saved by timing), fixed in round 6.

tools/vmem_audit.py replays the VMEM queue over each kernel's control-flow graph and reports any
instruction that touches an in-flight asm load's registers before the wait that names them. The
product must have none; the round-5 variant must be caught (the check has teeth)."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

pytestmark = pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="needs hipcc (gfx950 cross-compile)")


def _kernels(path):
    import vmem_audit as V
    return {n: lines for n, lines in V.parse_functions(path).items() if "bc_forward" in n}


@pytest.mark.parametrize("tu", ["bcfft_dmk", "bcfft_dm256", "bcfft_dm64k"])
def test_no_register_touch_of_inflight_asm_loads(tu, tmp_path):
    import vmem_audit as V
    ks = _kernels(V.compile_isa(tu, out_dir=str(tmp_path)))
    assert ks, tu
    bad = {}
    waited = 0
    for name, lines in ks.items():
        waited += sum(1 for s in lines if "bcfft-wait" in s)
        t_fwd, t_loop, _ = V.check(lines)
        if t_fwd or t_loop:
            bad[name] = (len(t_fwd), len(t_loop), [f"L{u.line + 1} {u.op} {u.args[:40]}" for _, u, *_ in (t_fwd + t_loop)[:3]])
    assert waited > 0, "no named waits: the kernels' wait_b no longer lists its registers (`; bcfft-wait`)"
    assert not bad, bad


def test_audit_catches_round5_late_dma_variant(tmp_path):
    """The re-created failing variant: the 16-token, no-bias instantiation (the one N = 4090 runs)
    has register copies of in-flight fragment registers inside its chunk loop."""
    import vmem_audit as V
    ks = _kernels(V.compile_isa("bcfft_dmk", ("-DBCFFT_DMK_LATE_DMA=1",), out_dir=str(tmp_path)))
    name = next(n for n in ks if "ILi16ELb0ELb0E" in n)
    _, t_loop, _ = V.check(ks[name])
    assert len(t_loop) > 0
    assert any(u.op.startswith("v_mov") for _, u, *_ in t_loop)
