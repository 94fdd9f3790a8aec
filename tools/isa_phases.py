"""Instruction mix per barrier-delimited segment of one kernel in a hipcc -save-temps .s file.
usage: python tools/isa_phases.py file.s kernel_substring"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2]
m = re.search(r"^(_Z\S*" + pat + r"\S*):", s, re.M)
i = m.start()
j = s.index(".Lfunc_end", i)
lines = [l.strip() for l in s[i:j].split("\n")]
segs = [[]]
for l in lines:
    if l.startswith(";MARK"):                 # -DBCFFT_MARKS phase markers
        segs.append([l])
        continue
    if not l or l.startswith(";") or l.startswith(".") or l.endswith(":"):
        continue
    op = l.split()[0]
    segs[-1].append(op)
    if op == "s_barrier":
        segs.append([])


def cls(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if "_dpp" in op:
        return "dpp"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "scratch_")):
        return "vmem"
    if op == "s_nop":
        return "nop"
    if op.startswith("s_waitcnt"):
        return "wait"
    return "salu"


for n, seg in enumerate(segs):
    c = collections.Counter(cls(o) for o in seg if not o.startswith(";"))
    tag = seg[0] if seg and seg[0].startswith(";MARK") else ""
    print(f"seg {n:2d} {tag:8s}: " + "  ".join(f"{k} {c[k]:4d}" for k in ("valu", "dpp", "mfma", "lds", "vmem", "nop", "wait", "salu")))
