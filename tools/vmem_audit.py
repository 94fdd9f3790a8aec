"""Static audit of the vector-memory (VMEM) ordering in the gfx950 code objects (CPU only).

The streamed-weight kernels issue some loads from inline asm (`buffer_load_dwordx4 v[..] ...` for
the B fragments, `buffer_load_dwordx4 ... lds` for the x DMA): the compiler does not count them in
its s_waitcnt bookkeeping, and it believes an asm load's destination registers hold their value as
soon as the asm statement ends. The program then relies on hand-placed `s_waitcnt vmcnt(N)`, and on
the compiler never touching those registers (copy, spill, reuse) before the covering wait.

This tool checks exactly that on the compiled ISA (`hipcc -S` output, per kernel):

  * every VMEM instruction (buffer_/global_/flat_/scratch_, loads, stores, LDS DMA, atomics) is an
    entry in an in-order queue; `s_waitcnt vmcnt(n)` retires all but the n youngest (gfx9: loads,
    stores and LDS-DMA count together, in issue order; MI355X_MICROARCH.md);
  * a dataflow over the kernel's control-flow graph keeps, per load still possibly in flight, the
    MINIMUM number of younger VMEM instructions over all paths (a load is retired by vmcnt(n) only
    if at least n younger ones were issued after it on every path): the conservative state;
  * any instruction that names a VGPR / AGPR of a possibly-in-flight load's destination (reads it:
    a stale value; writes it: the landing load overwrites the new value) is reported, with the load
    that is still in flight and the path-minimum count of younger operations.

Loads the compiler emitted itself are covered by its own waits (asm VMEM it cannot see only adds
younger operations, which makes its waits stricter), so every report is about hand-counted waits
or compiler register traffic around an asm load.

usage: python tools/vmem_audit.py file.s [kernel-substring]      (exit 1 when a hazard is found)
       python tools/vmem_audit.py --build [DEFS...]               (compile every product TU, audit all)
"""
import os
import re
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CAP = 64
VMEM_RE = re.compile(r"^(buffer|global|flat|scratch)_")
BRANCH_RE = re.compile(r"^s_(branch|cbranch_\w+)$")
REG_RE = re.compile(r"\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b")


def regs_of(text):
    out = set()
    for m in REG_RE.finditer(text):
        if m.group(1):
            f, lo, hi = m.group(1), int(m.group(2)), int(m.group(3))
            out.update((f, r) for r in range(lo, hi + 1))
        else:
            out.add((m.group(4), int(m.group(5))))
    return out


class Insn:
    __slots__ = ("idx", "line", "op", "args", "asm", "vmem", "lds_dma", "is_load", "dest", "touch", "vmcnt", "target")

    def __init__(self, idx, line, text, asm):
        self.idx, self.line, self.asm = idx, line, asm
        parts = text.split(None, 1)
        self.op = parts[0]
        self.args = parts[1] if len(parts) > 1 else ""
        a = self.args.split(";")[0]
        self.vmem = bool(VMEM_RE.match(self.op)) and not self.op.startswith(("buffer_wbl2", "buffer_inv"))
        self.lds_dma = self.vmem and re.search(r"\blds\b", a) is not None
        self.is_load = self.vmem and ("_load" in self.op or ("atomic" in self.op and re.search(r"\b(glc|sc0)\b", a)))
        ops = [o.strip() for o in a.split(",")]
        self.dest = regs_of(ops[0]) if (self.is_load and not self.lds_dma and ops) else set()
        self.touch = regs_of(a)
        self.vmcnt = None
        self.target = None
        if self.op == "s_waitcnt":
            m = re.search(r"vmcnt\((\d+)\)", a)
            if m:
                self.vmcnt = int(m.group(1))
            elif re.fullmatch(r"\s*0\s*", a):
                self.vmcnt = 0


def parse_functions(path):
    """{kernel name: [lines of its body]} from a hipcc -S listing."""
    funcs, cur, name = {}, None, None
    for ln in open(path):
        s = ln.rstrip("\n")
        m = re.match(r"^(_Z\w+):", s)
        if m:
            name, cur = m.group(1), []
            funcs[name] = cur
            continue
        if cur is not None:
            if s.startswith(".Lfunc_end") or s.strip().startswith(".size"):
                cur, name = None, None
                continue
            cur.append(s)
    return funcs


def build_cfg(lines):
    insns, labels, starts = [], {}, []
    in_asm = False
    for i, s in enumerate(lines):
        t = s.strip()
        if t.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if t.startswith(";;#ASMEND"):
            in_asm = False
            continue
        m = re.match(r"^(\.LBB\w+):", t)
        if m:
            labels[m.group(1)] = len(insns)
            starts.append(len(insns))
            continue
        if t.startswith("; %bb."):
            starts.append(len(insns))
            continue
        if not t or t.startswith((";", ".", "//")):
            continue
        insns.append(Insn(len(insns), i, t, in_asm))
    n = len(insns)
    succ = defaultdict(list)
    for ins in insns:
        if ins.op == "s_endpgm":
            continue
        if BRANCH_RE.match(ins.op):
            tgt = ins.args.split()[0]
            if tgt in labels:
                ins.target = labels[tgt]
                succ[ins.idx].append(labels[tgt])
            if ins.op != "s_branch" and ins.idx + 1 < n:
                succ[ins.idx].append(ins.idx + 1)
        elif ins.idx + 1 < n:
            succ[ins.idx].append(ins.idx + 1)
    return insns, succ


SOP_RE = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b")


def sregs(text):
    out = []
    for m in SOP_RE.finditer(text):
        if m.group(1):
            out += [int(r) for r in range(int(m.group(1)), int(m.group(2)) + 1)]
        else:
            out.append(int(m.group(3)))
    return out


def scalar_step(ins, consts):
    """Updates the known scalar constants in place for one instruction; returns (branch taken
    feasible, fall-through feasible). Tracks s_mov_b32/b64 of 0 / -1, vcc from s_and(n2)_b64 vcc,
    exec, s[..] and scc from s_cmp_lg/eq_u64 s[..], 0; anything else that writes a tracked
    register (or vcc / scc) forgets it."""
    op, a = ins.op, ins.args.split(";")[0]
    ops = [o.strip() for o in a.split(",")]
    taken, fall = True, True

    def known(regs):
        vals = [consts.get(("s", r)) for r in regs]
        return None if (not regs or any(v is None for v in vals)) else all(v == -1 for v in vals) and "ones" or (
            "zero" if all(v == 0 for v in vals) else "mixed")

    if op.startswith("s_cbranch_"):
        cond = op[len("s_cbranch_"):]
        v = consts.get(("vcc",)) if cond in ("vccz", "vccnz") else consts.get(("scc",)) if cond in ("scc0", "scc1") else None
        if v is not None:
            t = {"vccz": v == 0, "vccnz": v == 1, "scc0": v == 0, "scc1": v == 1}[cond]
            taken, fall = t, not t
        return taken, fall
    return _scalar_rest(ins, consts, known)


def branch_facts(ins, consts, taken):
    """The facts a conditional branch establishes on the edge it takes (taken=True) or falls
    through: vcc computed as s_and(n2)_b64 vcc, exec, s[a:b] from a uniform condition s[a:b]
    (all lanes set or none) tells whether s[a:b] is zero; recorded as ("flag", a) -> 0 / 1, so a
    later test of the same, unmodified s[a:b] is decided (the compiler's `if (c) A; ...; if (!c) B`
    over one condition)."""
    cond = ins.op[len("s_cbranch_"):]
    sym = consts.get(("vccsym",))
    if cond not in ("vccz", "vccnz") or sym is None:
        return
    reg, neg = sym
    vcc_nz = (cond == "vccnz") == taken             # the edge implies vcc != 0
    flag_nz = vcc_nz != neg                          # s_and: vcc != 0 iff s != 0; s_andn2: iff s == 0
    consts[("flag", reg)] = 1 if flag_nz else 0


def _scalar_rest(ins, consts, known):
    """scalar_step for the non-branch instructions."""
    op, a = ins.op, ins.args.split(";")[0]
    ops = [o.strip() for o in a.split(",")]
    taken, fall = True, True
    if op in ("s_branch", "s_waitcnt", "s_barrier", "s_nop", "s_setprio", "s_endpgm") or not ops or not ops[0]:
        return taken, fall
    dst = ops[0]
    if op in ("s_mov_b64", "s_mov_b32") and dst.startswith("s") and len(ops) == 2 and ops[1] in ("0", "-1"):
        for r in sregs(dst):
            consts[("s", r)] = int(ops[1])
        return taken, fall
    if op in ("s_and_b64", "s_andn2_b64") and dst == "vcc" and len(ops) == 3 and ops[1] == "exec":
        regs = sregs(ops[2])
        k = known(regs)
        consts.pop(("scc",), None)
        consts.pop(("vccsym",), None)
        if k is None and regs and ("flag", regs[0]) in consts:
            k = "ones" if consts[("flag", regs[0])] else "zero"
        if k in ("ones", "zero"):
            nz = (k == "ones") if op == "s_and_b64" else (k == "zero")
            consts[("vcc",)] = 1 if nz else 0
        else:
            consts.pop(("vcc",), None)
            if regs:
                consts[("vccsym",)] = (regs[0], op == "s_andn2_b64")
        return taken, fall
    if op in ("s_cmp_lg_u64", "s_cmp_eq_u64") and len(ops) == 2 and ops[1] == "0":
        k = known(sregs(ops[0]))
        if k in ("ones", "zero"):
            nz = k == "ones"
            consts[("scc",)] = int(nz if op == "s_cmp_lg_u64" else not nz)
        else:
            consts.pop(("scc",), None)
        return taken, fall
    # generic: forget what this instruction may write (its first operand, vcc, scc); compares
    # (s_cmp*, s_bitcmp*) write only scc
    if op.startswith(("s_cmp", "s_bitcmp")):
        consts.pop(("scc",), None)
        return taken, fall
    for r in sregs(dst):
        consts.pop(("s", r), None)
        consts.pop(("flag", r), None)
        sym = consts.get(("vccsym",))
        if sym and sym[0] == r:
            consts.pop(("vccsym",), None)
    if "vcc" in dst or op.startswith("v_cmp") or op.startswith("v_add_co") or op.startswith("v_sub_co"):
        consts.pop(("vcc",), None)
        consts.pop(("vccsym",), None)
    if op.startswith("s_"):
        consts.pop(("scc",), None)
    return taken, fall


def audit(lines, forward=False):
    """Returns (hazards, orphans, asm VMEM count). Forward dataflow of {load: min younger VMEM count
    over all paths} per instruction; then, per asm load L with destination registers:
      * its consumers are the asm waits that name its registers (`; bcfft-wait <regs>`, the
        kernels' wait_b); a consumer reached with L in flight must retire it (>= N younger VMEM
        instructions on every path, for its vmcnt(N)), else the wait does not cover the load;
      * an instruction that touches L's registers while L may be in flight, on a path that goes on
        to one of L's consumers, is a hazard (the compiler read a stale value, or wrote a register
        the landing load then overwrites);
      * a touch on a path that never reaches a consumer is counted as an orphan: either the path
        is infeasible (e.g. the next chunk's fragments are loaded only while there is a next chunk,
        `cn >= 0`, and the path skips that chunk) or the load is never waited for at all."""
    insns, succ = build_cfg(lines)
    if forward:                                     # one loop iteration: no back edges
        succ = defaultdict(list, {i: [j for j in js if j > i] for i, js in succ.items()})
    if not insns:
        return [], 0, 0
    # Path states carry a few known scalar constants, so that the compiler's if / else over a
    # uniform flag (`s_mov_b64 s[4:5], -1; s_and_b64 vcc, exec, c; s_cbranch_vccz A; <then>;
    # s_mov_b64 s[4:5], 0; A: s_andn2_b64 vcc, exec, s[4:5]; s_cbranch_vccnz B; <else>`) is not
    # walked through neither branch (a path on which the x DMA of neither branch issues).
    # state_in[i] = {consts: {load: min younger count}}, consts a frozenset of (register, value).
    consumers = [x for x in insns if x.asm and x.op == "s_waitcnt" and "bcfft-wait" in x.args]
    cregs = {x.idx: regs_of(x.args.split("bcfft-wait", 1)[1]) for x in consumers}
    state_in = {0: {frozenset(): {}}}
    work = [(0, frozenset())]
    while work:
        i, key = work.pop()
        st = dict(state_in[i][key])
        consts = dict(key)
        ins = insns[i]
        if ins.vmcnt is not None:
            st = {k: c for k, c in st.items() if c < ins.vmcnt}
        if i in cregs:                              # the wait that names a load's registers ends its
            st = {k: c for k, c in st.items() if not (insns[k].dest & cregs[i])}   # window (its count: below)
        if ins.vmem:
            st = {k: min(c + 1, CAP) for k, c in st.items()}
            if ins.dest and ins.asm:
                st[i] = 0
        taken_ok, fall_ok = scalar_step(ins, consts)
        nkey = frozenset(consts.items())
        for j in succ[i]:
            if BRANCH_RE.match(ins.op) and ins.op != "s_branch":
                ok = (j == ins.target and taken_ok) or (j == i + 1 and fall_ok)
                if not ok:
                    continue
                ec = dict(consts)
                branch_facts(ins, ec, j == ins.target)
                nkey = frozenset(ec.items())
            bucket = state_in.setdefault(j, {})
            if len(bucket) >= 16 and nkey not in bucket:
                kk = frozenset()                    # too many splits: forget the constants
            else:
                kk = nkey
            old = bucket.get(kk)
            if old is None:
                new = dict(st)
            else:
                new = dict(old)
                for k, c in st.items():
                    new[k] = min(new.get(k, CAP), c)
            if old != new:
                bucket[kk] = new
                work.append((j, kk))
    # merge the per-constant states: min over all path classes
    merged = {}
    for i, bucket in state_in.items():
        m = {}
        for stt in bucket.values():
            for k, c in stt.items():
                m[k] = min(m.get(k, CAP), c)
        merged[i] = m
    state_in = merged
    pred = defaultdict(list)
    for i, js in succ.items():
        for j in js:
            pred[j].append(i)
    hazards, orphans = [], 0
    for ld in insns:
        if not (ld.asm and ld.dest):
            continue
        cons = [x for x in consumers if cregs[x.idx] & ld.dest]
        # instructions from which a consumer of ld is reachable without re-issuing ld
        back, stack = set(), [x.idx for x in cons]
        while stack:
            x = stack.pop()
            if x in back:
                continue
            back.add(x)
            stack.extend(p for p in pred[x] if p != ld.idx)
        for x in cons:
            c = state_in.get(x.idx, {}).get(ld.idx)
            if c is not None and c < x.vmcnt:
                hazards.append((ld, x, c, sorted(ld.dest), "wait does not retire the load"))
        for ins in insns:
            st = state_in.get(ins.idx)
            if not st or ld.idx not in st or ins.idx == ld.idx or ins.idx in cregs:
                continue
            c = st[ld.idx]
            if ins.vmcnt is not None and c >= ins.vmcnt:
                continue
            ov = ld.dest & (ins.touch - ins.dest if ins.is_load else ins.touch)
            if not ov:
                continue
            if ins.idx in back or not cons:
                # no wait names this load's registers at all: the compiler renamed them between the
                # load and the wait meant for it (a copy / move of the in-flight registers), so every
                # touch is a hazard (round 6: a dm8 variant with prologue-loaded fragments did this)
                hazards.append((ld, ins, c, sorted(ov), "touched in flight"))
            else:
                orphans += 1
    n_asm = sum(1 for x in insns if x.vmem and x.asm)
    return hazards, orphans, n_asm


def steady_loop(insns, succ):
    """Instruction set of the smallest natural loop holding both an asm load with register
    destinations and a consumer wait: the streamed-weight kernels' chunk / step loop."""
    pred = defaultdict(list)
    for i, js in succ.items():
        for j in js:
            pred[j].append(i)
    best = set()
    for i, js in succ.items():
        for h in js:
            if h > i:
                continue
            body, stack = {h}, [i]
            while stack:
                x = stack.pop()
                if x in body:
                    continue
                body.add(x)
                stack.extend(pred[x])
            if (any(insns[x].asm and insns[x].dest for x in body)
                    and any(insns[x].asm and "bcfft-wait" in insns[x].args for x in body)
                    and (not best or len(body) < len(best))):
                best = body
    return best


def check(lines):
    """The two verdicts the tests assert, per kernel (both free of the dataflow's infeasible-path
    reports):
      * within one iteration (no back edges): no instruction touches the registers of an asm load
        before a wait that names and retires them;
      * across iterations: no instruction inside the steady-state loop touches them while the
        load may be in flight.
    Returns (within-iteration touches, steady-loop touches, unretired-wait reports (information:
    the path-insensitive count can take a loop that always runs twice through once))."""
    fwd, _, _ = audit(lines, forward=True)
    full, _, _ = audit(lines)
    insns, succ = build_cfg(lines)
    loop = steady_loop(insns, succ)
    t_fwd = [h for h in fwd if h[4] == "touched in flight"]
    t_loop = [h for h in full if h[4] == "touched in flight" and h[1].idx in loop]
    waits = [h for h in full if h[4] != "touched in flight"]
    return t_fwd, t_loop, waits


def fmt_regs(rs):
    by = defaultdict(list)
    for f, r in rs:
        by[f].append(r)
    return " ".join(f"{f}{min(v)}..{max(v)}" if len(v) > 1 else f"{f}{v[0]}" for f, v in by.items())


def audit_file(path, filt=None, verbose=True):
    """check() per kernel of a listing; returns the number of register touches in flight."""
    bad = 0
    for name, lines in parse_functions(path).items():
        if filt and filt not in name:
            continue
        t_fwd, t_loop, waits = check(lines)
        n_asm = sum(1 for s in lines if "buffer_load" in s) if verbose else 0
        if verbose:
            print(f"{os.path.basename(path)} {name[:80]}: {len(t_fwd)} within-iteration / {len(t_loop)} "
                  f"steady-loop register touches in flight; {len(waits)} unretired-wait reports (information)")
        for ld, use, c, ov, why in (t_fwd + t_loop)[:12]:
            print(f"    {why}: load L{ld.line + 1} {ld.op} {ld.args[:60]}")
            print(f"      at L{use.line + 1} {'asm ' if use.asm else ''}{use.op} {use.args[:70]}  "
                  f"[{fmt_regs(ov)}; >= {c} younger VMEM on every path]")
        bad += len(t_fwd) + len(t_loop)
    return bad


# translation units that issue VMEM loads into registers from inline asm (the streamed-weight kernels)
ASM_LOAD_TUS = ("bcfft_dmk", "bcfft_dm256", "bcfft_dm64k")


def compile_isa(tu, defs=(), out_dir="/tmp/vmem_audit"):
    """hipcc -S of one product translation unit for gfx950 (the product's flags); returns the path."""
    os.makedirs(out_dir, exist_ok=True)
    tag = "".join(d.replace("-D", "_").replace("=", "") for d in defs)
    s = os.path.join(out_dir, f"{tu}{tag}.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                    f"-I{ROOT}/include", "-ffp-contract=fast", "-fno-slp-vectorize", "--cuda-device-only",
                    "-S", *defs, os.path.join(ROOT, "llama-fft_amd", "csrc", f"{tu}.hip"), "-o", s],
                   check=True, stderr=subprocess.DEVNULL)
    return s


def build_and_audit(defs):
    return sum(audit_file(compile_isa(tu, defs)) for tu in ASM_LOAD_TUS)


if __name__ == "__main__":
    if sys.argv[1] == "--build":
        nbad = build_and_audit(sys.argv[2:])
    else:
        nbad = audit_file(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
    print(f"total hazards: {nbad}")
    sys.exit(1 if nbad else 0)
