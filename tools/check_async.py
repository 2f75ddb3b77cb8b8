"""Heuristic hazard scan of a hipcc -S dump: flags instructions that READ a
VGPR still being written by an outstanding global load (i.e. before the
s_waitcnt vmcnt that retires it), following the layout order of each kernel
(branches are not followed; loop back-edges are ignored).

usage: python tools/check_async.py file.s kernel_substring [...]"""
import re
import sys


def regs(tok):
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"v(\d+)", tok)
    return {int(m.group(1))} if m else set()


def scan(lines, name):
    out = []  # outstanding VMEM ops: (dest regs, line)
    issues = 0
    for ln in lines:
        t = ln.split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":"):
            if t.startswith(".LBB") or t.endswith(":"):
                pass
            continue
        op = t.split()[0]
        ops = [o.strip() for o in t[len(op):].split(",")]
        if op in ("s_branch", "s_setpc_b64"):
            out = []  # the next block in layout order is reached from elsewhere
            continue
        if op == "s_waitcnt":
            m = re.search(r"vmcnt\((\d+)\)", t)
            if m:
                n = int(m.group(1))
                out = out[len(out) - n:] if n < len(out) else out
                if n == 0:
                    out = []
            continue
        if op.startswith(("global_load", "buffer_load", "scratch_load")):
            srcs = set().union(*(regs(o) for o in ops[1:])) if len(ops) > 1 else set()
            for d, l0 in out:
                if d & srcs:
                    issues += 1
                    print(f"  [{name}] address reads in-flight reg: {t}   (load: {l0})")
            out.append((regs(ops[0]), t))
            continue
        if op.startswith(("global_store", "buffer_store", "scratch_store")):
            srcs = set().union(*(regs(o) for o in ops))
            for d, l0 in out:
                if d & srcs:
                    issues += 1
                    print(f"  [{name}] store reads in-flight reg: {t}   (load: {l0})")
            out.append((set(), t))
            continue
        # generic instruction: operands after the first are sources (first is dst),
        # except for v_mfma where all but the first are sources too
        srcs = set()
        for o in ops[1:]:
            srcs |= regs(o)
        dst = regs(ops[0]) if ops else set()
        for d, l0 in out:
            if d & srcs:
                issues += 1
                print(f"  [{name}] reads in-flight reg: {t}   (load: {l0})")
        # a write to an in-flight destination is also a hazard (WAW)
        for d, l0 in out:
            if d & dst and not op.startswith("s_"):
                issues += 1
                print(f"  [{name}] overwrites in-flight reg: {t}   (load: {l0})")
    return issues


src = open(sys.argv[1]).read().splitlines()
total = 0
for pat in sys.argv[2:]:
    starts = [i for i, l in enumerate(src) if pat in l and l.split(";")[0].rstrip().endswith(":") and not l.startswith("\t")]
    for st in starts:
        en = next(i for i in range(st, len(src)) if "s_endpgm" in src[i])
        name = src[st].split(":")[0][:60]
        n = scan(src[st:en], name)
        print(f"{name}: {n} potential hazards")
        total += n
sys.exit(1 if total else 0)
