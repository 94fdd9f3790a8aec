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


def test_audit_reports_a_load_whose_registers_were_renamed():
    """Round 6: a variant that loaded the stationary fragments by asm in the prologue and waited for
    them inside the loop got its registers moved by hipcc between the two (the wait named other
    registers than the loads wrote). The audit once counted such touches as orphans (no wait names
    the load); every touch of an unnamed in-flight load is a hazard now. Synthetic listing."""
    import vmem_audit as V
    lines = [
        "\t;;#ASMSTART",
        "\tbuffer_load_dwordx4 v[0:3], v8, s[4:7], 0 offen",
        "\t;;#ASMEND",
        "\tv_mov_b64_e32 v[4:5], v[0:1]",        # the compiler's copy of the in-flight registers
        "\tv_mov_b64_e32 v[6:7], v[2:3]",
        "\t;;#ASMSTART",
        "\ts_waitcnt vmcnt(0) ; bcfft-wait v[4:7]",
        "\t;;#ASMEND",
        "\ts_endpgm",
    ]
    t_fwd, t_loop, _ = V.check(lines)
    assert len(t_fwd) >= 2
