"""Heuristic hazard scan of a hipcc -S dump: flags instructions that READ a
VGPR still being written by an outstanding global load (i.e. before the
s_waitcnt vmcnt that retires it), following the layout order of each kernel
(branches are not followed; loop back-edges are ignored).

The hazard: ``gload*_async`` (cfsd_common.h) issues a global load in inline
asm, hidden from hipcc's waitcnt bookkeeping, and ``vm_wait*`` retires it by
count; if hipcc schedules a read of the destination (or a copy of it) before
that wait, the kernel silently uses stale data.  ``build()`` runs this over
every kernel of every source (``make -C craniofacialsd-vae_amd/csrc check``),
so a compiler update that reintroduces the hazard fails the build.

usage: python tools/check_async.py file.s kernel_substring [...]
       python tools/check_async.py --all file.s [...]   (every kernel)"""
import re
import sys


def regs(tok):
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"v(\d+)", tok)
    return {int(m.group(1))} if m else set()


def scan(lines, name, log=print):
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
                    log(f"  [{name}] address reads in-flight reg: {t}   (load: {l0})")
            out.append((regs(ops[0]), t))
            continue
        if op.startswith(("global_store", "buffer_store", "scratch_store")):
            srcs = set().union(*(regs(o) for o in ops))
            for d, l0 in out:
                if d & srcs:
                    issues += 1
                    log(f"  [{name}] store reads in-flight reg: {t}   (load: {l0})")
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
                log(f"  [{name}] reads in-flight reg: {t}   (load: {l0})")
        # a write to an in-flight destination is also a hazard (WAW)
        for d, l0 in out:
            if d & dst and not op.startswith("s_"):
                issues += 1
                log(f"  [{name}] overwrites in-flight reg: {t}   (load: {l0})")
    return issues


def kernels(src, pats=None):
    """(name, first line, end line) of every kernel body in a -S dump whose
    label contains one of ``pats`` (all kernels when ``pats`` is None)."""
    for i, l in enumerate(src):
        if l.startswith("\t") or not l.split(";")[0].rstrip().endswith(":"):
            continue
        if pats is None and not l.startswith("_Z"):
            continue
        if pats is not None and not any(p in l for p in pats):
            continue
        en = next((j for j in range(i, len(src)) if "s_endpgm" in src[j]), None)
        if en is not None:
            yield src[i].split(":")[0], i, en


def main(argv, log=print):
    if argv and argv[0] == "--all":
        files, pats = argv[1:], None
    else:
        files, pats = argv[:1], argv[1:]
    total, n_k = 0, 0
    for fn in files:
        src = open(fn).read().splitlines()
        for name, st, en in kernels(src, pats):
            n = scan(src[st:en], name[:60], log)
            n_k += 1
            if n or pats is not None:
                log(f"{name[:60]}: {n} potential hazards")
            total += n
    log(f"check_async: {n_k} kernels in {len(files)} file(s), {total} potential hazards")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
