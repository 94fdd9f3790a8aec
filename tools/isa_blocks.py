"""Static instruction mix per basic block of one kernel in a hipcc -S listing.

usage: python tools/isa_blocks.py k.s <kernel-substring> [--min N]
Prints, per block: label, VALU / MFMA / SALU / DS / VMEM / waitcnt counts and the branch
targets, so loops (backward branches) and their bodies can be costed by hand.
"""
import re
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and pat in l)
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, cur = [], {"label": "entry", "n": {}, "br": []}
    for l in lines[start + 1:end]:
        s = l.strip()
        m = re.match(r"^(\.LBB\S+):", s)
        if m:
            blocks.append(cur)
            cur = {"label": m.group(1), "n": {}, "br": []}
            continue
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        if op.startswith("v_mfma"):
            k = "mfma"
        elif op.startswith("v_"):
            k = "valu"
        elif op.startswith("s_waitcnt"):
            k = "wait"
        elif op.startswith("s_barrier"):
            k = "bar"
        elif op.startswith("s_cbranch") or op == "s_branch":
            cur["br"].append(s.split()[-1])
            k = "salu"
        elif op.startswith("s_"):
            k = "salu"
        elif op.startswith("ds_"):
            k = "ds"
        elif op.startswith(("global_", "buffer_", "flat_")):
            k = "vmem"
        else:
            k = "other"
        cur["n"][k] = cur["n"].get(k, 0) + 1
    blocks.append(cur)
    tot = {}
    for b in blocks:
        n = b["n"]
        for k, v in n.items():
            tot[k] = tot.get(k, 0) + v
        if sum(n.values()) >= int(sys.argv[4]) if len(sys.argv) > 4 else True:
            print(f"{b['label']:14s} valu {n.get('valu',0):5d} mfma {n.get('mfma',0):4d} salu {n.get('salu',0):4d} "
                  f"ds {n.get('ds',0):4d} vmem {n.get('vmem',0):4d} wait {n.get('wait',0):3d} bar {n.get('bar',0):2d} "
                  f"-> {' '.join(b['br'])}")
    print("total", tot)


if __name__ == "__main__":
    main()
