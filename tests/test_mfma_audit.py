"""CPU check of the gfx950 code objects for MFMA SrcC chains across opcodes (tools/mfma_audit.py).

On gfx950 an MFMA that reads as SrcC the result of an MFMA of another opcode (f16 <-> fp8_bf8)
issued fewer than ~6 instructions before reads a stale C in every lane (tools/probe/srcc.hip,
profiles/r06j_mfma_srcc_chain_probe.txt), and hipcc inserts no wait states for the pair. The
precise engine's residual MFMAs are the only cross-opcode chains in the product; xdl_gap
(bcfft_dm.hip) separates them. This test compiles every product translation unit and fails on
any such pair, and checks that the audit does see the pair in the round-5 form of the kernel."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

pytestmark = pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="needs hipcc (gfx950 cross-compile)")


def test_no_cross_opcode_srcc_chain_in_product():
    import mfma_audit as M
    found = M.audit_tu("bcfft_dm", verbose=False)
    assert not found, {k[:80]: v[:3] for k, v in found.items()}


def test_audit_sees_an_unseparated_chain(tmp_path):
    """The same kernel with xdl_gap emptied (the round-5 form): the audit must report pairs."""
    import subprocess
    import mfma_audit as M
    import vmem_audit as V
    src = open(os.path.join(ROOT, "llama-fft_amd", "csrc", "bcfft_dm.hip")).read()
    old = 'asm volatile("s_nop 7" : "+v"(acc));'
    assert src.count(old) == 1
    patched = tmp_path / "bcfft_dm_nogap.hip"
    patched.write_text(src.replace(old, 'asm volatile("" : "+v"(acc));'))
    out = tmp_path / "nogap.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                    f"-I{ROOT}/include", f"-I{ROOT}/llama-fft_amd/csrc", "-ffp-contract=fast", "-fno-slp-vectorize",
                    "--cuda-device-only", "-S", str(patched), "-o", str(out)], check=True, stderr=subprocess.DEVNULL)
    bad = {n: M.check(lines) for n, lines in V.parse_functions(str(out)).items()}
    assert any(bad.values())
