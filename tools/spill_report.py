"""Where does a kernel spill? Counts scratch ops per barrier-delimited segment of a hipcc -save-temps .s."""
import collections
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else "bc_forward_stat_kernel"
for m in re.finditer(r"^(_Z\S*" + pat + r"\S*):", s, re.M):
    name = m.group(1)
    i = m.start()
    j = s.index(".Lfunc_end", i)
    k = s[i:j].split("\n")
    sc = [n for n, l in enumerate(k) if "scratch_" in l]
    bar = [n for n, l in enumerate(k) if "s_barrier" in l]
    hist = collections.Counter(sum(1 for b in bar if b < n) for n in sc)
    vg = re.search(r"\.vgpr_count:\s+(\d+)", s[j:j + 20000])
    print(f"{name[:70]:70s} lines {len(k):5d} scratch {len(sc):4d} by segment {sorted(hist.items())}")
