"""Static audit of MFMA accumulation chains across opcodes in the gfx950 code objects (CPU only).

Finding (round 6, tools/probe/srcc.hip, profiles/r06j_mfma_srcc_chain_probe.txt): an MFMA that
reads as SrcC the result of an earlier MFMA of ANOTHER opcode (v_mfma_f32_16x16x32_f16 ->
v_mfma_f32_16x16x32_fp8_bf8, or the reverse) reads a stale C in every lane when 0-3 independent
instructions separate the two, and the right one at 6. The same pair of one opcode (an
accumulation chain) is forwarded back to back. hipcc inserts no wait states for either pair, so
the cross-opcode chain is left to the schedule: the precise engine's 16-bit-x and 16-bit-bias
instantiations computed wrong values from exactly this.

This tool lists, per kernel, every MFMA whose SrcC registers were last written by an MFMA of a
different opcode fewer than MIN_GAP wait states before (an instruction counts 1, `s_nop N` counts
N + 1), scanning the `hipcc -S` listing in program order. Program order covers the unrolled
straight-line chains these kernels build; a chain across a loop's back edge would need the CFG
(tools/vmem_audit.py has one), and none of the kernels accumulate across one.

usage: python tools/mfma_audit.py [TU ...]      (default: every product TU; exit 1 on a finding)
"""
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import vmem_audit as V  # noqa: E402

MIN_GAP = 6
MFMA_RE = re.compile(r"^\s*(v_mfma_\w+)\s+(.*)$")
REG_RE = re.compile(r"\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b")
NOP_RE = re.compile(r"^\s*s_nop\s+(\d+)")
PRODUCT_TUS = ("bcfft_dm", "bcfft_dm8", "bcfft_dm64", "bcfft_dmk", "bcfft_dmg", "bcfft_dm256", "bcfft_dm64k",
               "bcfft_dm64g", "bcfft_dmm", "bcfft_sn", "bcfft_stat", "bcfft_kernels", "bcfft_grad", "bcfft_prep")


def _regs(operand):
    m = REG_RE.search(operand)
    if not m:
        return set()
    if m.group(1):
        return {(m.group(1), r) for r in range(int(m.group(2)), int(m.group(3)) + 1)}
    return {(m.group(4), int(m.group(5)))}


def check(lines):
    """[(line, opcode, src opcode, gap)] of the cross-opcode SrcC reads closer than MIN_GAP."""
    last = {}                          # register -> (opcode, wait-state clock of the write)
    clock = 0
    bad = []
    for i, ln in enumerate(lines):
        s = ln.split(";")[0].strip()
        if not s or s.endswith(":") or s.startswith("."):
            continue
        m = NOP_RE.match(s)
        if m:
            clock += int(m.group(1)) + 1
            continue
        clock += 1
        m = MFMA_RE.match(s)
        if not m:
            continue
        op, args = m.group(1), [a.strip() for a in m.group(2).split(",")]
        if len(args) >= 4:
            for r in _regs(args[3]):
                if r in last and last[r][0] != op and clock - last[r][1] - 1 < MIN_GAP:
                    bad.append((i + 1, op, last[r][0], clock - last[r][1] - 1))
                    break
        for r in _regs(args[0]):
            last[r] = (op, clock)
    return bad


def audit_tu(tu, verbose=True):
    path = V.compile_isa(tu, out_dir="/tmp/mfma_audit")
    found = {}
    for name, lines in V.parse_functions(path).items():
        bad = check(lines)
        if bad:
            found[name] = bad
            if verbose:
                print(f"{tu}: {name[:90]}: {len(bad)} cross-opcode SrcC reads closer than {MIN_GAP}")
                for ln, op, src, gap in bad[:4]:
                    print(f"    L{ln} {op} reads C of {src} after {gap} wait states")
    return found


def main():
    tus = sys.argv[1:] or PRODUCT_TUS
    n = sum(len(audit_tu(tu)) for tu in tus)
    print(f"{len(tus)} translation units: {n} kernels with a cross-opcode SrcC chain closer than {MIN_GAP}")
    sys.exit(1 if n else 0)


if __name__ == "__main__":
    main()
