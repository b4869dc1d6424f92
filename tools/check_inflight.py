"""Static check of the inline-asm load pipeline (build infrastructure).

Phase B of the split kernel issues `global_load_dwordx4 ... nt` from inline asm
and waits for it with explicitly counted `s_waitcnt vmcnt(N)` (hipcc would
drain vmcnt to 0 inside the loop otherwise).  The compiler believes the asm's
destination registers hold their value as soon as the asm is issued, so
nothing stops it from copying, spilling or reusing them before the wait -- it
would then read or clobber a register the load has not filled yet.  Seen once:
a `v_mov_b64` of a stage register, hoisted above its wait, gave nondeterministic
checks in one launch shape.

This script builds each kernel's control-flow graph from the device assembly
(`make asm`), propagates the queue of outstanding vector-memory operations
along it to a fixed point (vmcnt counts in issue order; a join keeps, per
queue position from the youngest, the union of what may be there), and
reports any instruction that names a register of an inline-asm load that may
still be outstanding.  `make` runs it on every build of the library.

    python tools/check_inflight.py [build/asm/checksummer-gfx950.s]
"""
import re
import sys

VMEM = re.compile(r"^(global_|buffer_|flat_|scratch_)(load|store|atomic)")
REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
LABEL = re.compile(r"^(\.LBB\w+|\.Ltmp\w+):")
BRANCH = re.compile(r"^(s_branch|s_cbranch_\w+)\s+(\S+)")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return frozenset(out)


def kernels(lines):
    """(name, [(line no, instruction text, in_asm)]) per function body."""
    name, body, in_asm = None, [], False
    for no, line in enumerate(lines, 1):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            name, body, in_asm = m.group(1), [], False
            continue
        if name is None:
            continue
        if line.startswith(".Lfunc_end"):
            yield name, body
            name = None
            continue
        if ";;#ASMSTART" in line:
            in_asm = True
            continue
        if ";;#ASMEND" in line:
            in_asm = False
            continue
        s = line.split(";")[0].strip()
        if not s or (s.startswith(".") and not LABEL.match(s)):
            continue
        body.append((no, s, in_asm))


def blocks(body):
    """Split into basic blocks: [(label or None, [insts], [successor labels], falls_through)]."""
    out, cur, label = [], [], None
    for no, s, in_asm in body:
        m = LABEL.match(s)
        if m:
            if cur or label is not None:
                out.append([label, cur])
            label, cur = m.group(1), []
            continue
        cur.append((no, s, in_asm))
        if BRANCH.match(s) or s.startswith("s_endpgm") or s.startswith("s_setpc"):
            out.append([label, cur])
            label, cur = None, []
    if cur or label is not None:
        out.append([label, cur])
    succ = []
    for i, (label, insts) in enumerate(out):
        last = insts[-1][1] if insts else ""
        nxt = [i + 1] if i + 1 < len(out) else []
        m = BRANCH.match(last)
        if m:
            tgt = [j for j, b in enumerate(out) if b[0] == m.group(2)]
            succ.append(tgt + ([] if m.group(1) == "s_branch" else nxt))
        elif last.startswith("s_endpgm") or last.startswith("s_setpc"):
            succ.append([])
        else:
            succ.append(nxt)
    return out, succ


def join(a, b):
    """Queues are tuples of frozensets, youngest last; align at the youngest end."""
    n = max(len(a), len(b))
    a = (frozenset(),) * (n - len(a)) + a
    b = (frozenset(),) * (n - len(b)) + b
    return tuple(x | y for x, y in zip(a, b))


def step(q, s, in_asm, report):
    if s.startswith("s_waitcnt"):
        m = re.search(r"vmcnt\((\d+)\)", s)
        if m:
            n = int(m.group(1))
            q = q[len(q) - n:] if len(q) > n else q
        return q
    pending = frozenset().union(*q) if q else frozenset()
    hit = regs(s) & pending
    if hit:
        report(s, hit)
    if VMEM.match(s):
        ops = s.split(None, 1)[1] if len(s.split(None, 1)) > 1 else ""
        dest = regs(ops.split(",")[0]) if (in_asm and "load" in s and "_lds_" not in s) else frozenset()
        q = q + (dest,)
        if len(q) > 64:                  # vmcnt saturates; older ones are long done
            q = q[-64:]
    return q


SPAIR = re.compile(r"^(s\[\d+:\d+\]|vcc)$")


def consts_step(c, s):
    """Known 64-bit SGPR-pair constants (s_mov_b64 -1/0, and vcc derived from
    them by `s_and(n2)_b64 vcc, exec, pair`), enough to prune the infeasible
    edges of hipcc's loop-exit idiom (`s_mov_b64 s[0:1], -1` ...
    `s_andn2_b64 vcc, exec, s[0:1]` / `s_cbranch_vccnz`)."""
    parts = s.replace(",", " ").split()
    if len(parts) < 2:
        return c
    op, dst = parts[0], parts[1]
    c = dict(c)
    # exec: "full" (every lane, as at kernel entry) or unknown; pairs that hold
    # a saved full exec restore it with s_or_b64 exec, exec, pair
    if op in ("s_and_saveexec_b64", "s_or_saveexec_b64", "s_andn2_saveexec_b64", "s_xor_saveexec_b64"):
        full = c.get("exec") == "full"
        c.pop("exec", None)
        c.pop("saved:" + dst, None)
        c.pop(dst, None)
        if full:
            c["saved:" + dst] = 1
        return c
    if dst == "exec":
        if op == "s_or_b64" and len(parts) == 4 and parts[2] == "exec" and "saved:" + parts[3] in c:
            c["exec"] = "full"
        elif op == "s_mov_b64" and len(parts) == 3 and (parts[2] == "-1" or "saved:" + parts[2] in c):
            c["exec"] = "full"
        else:
            c.pop("exec", None)
        return c
    if SPAIR.match(dst):
        c.pop("saved:" + dst, None)
    if op == "s_mov_b64" and SPAIR.match(dst) and len(parts) == 3 and parts[2] == "exec" and c.get("exec") == "full":
        c["saved:" + dst] = 1
        return c
    if op == "s_mov_b64" and SPAIR.match(dst) and len(parts) == 3 and parts[2] in ("-1", "0"):
        c[dst] = int(parts[2])
        return c
    if op in ("s_and_b64", "s_andn2_b64") and dst == "vcc" and len(parts) == 4 and parts[2] == "exec":
        v = c.get(parts[3])
        c.pop("vcc", None)
        if v is not None:
            if (op == "s_andn2_b64" and v == -1) or (op == "s_and_b64" and v == 0):
                c["vcc"] = 0
        return c
    # anything else that writes a pair (or vcc, implicitly by VOPC) forgets it
    if SPAIR.match(dst):
        c.pop(dst, None)
    if op.startswith("v_cmp") or "vcc" in parts[1:]:
        c.pop("vcc", None)
    if op.startswith("v_cmpx") or "exec" in parts[1:2]:
        c.pop("exec", None)
    return c


def feasible_succ(c, last, targets, fall):
    m = BRANCH.match(last)
    if m and m.group(1) in ("s_cbranch_vccnz", "s_cbranch_vccz") and c.get("vcc") == 0:
        return fall if m.group(1) == "s_cbranch_vccnz" else targets
    # where exec is known full (wave-uniform code), exec branches are decided
    if m and m.group(1) == "s_cbranch_execnz" and c.get("exec") == "full":
        return targets
    if m and m.group(1) == "s_cbranch_execz" and c.get("exec") == "full":
        return fall
    return targets + fall


def check_kernel(name, body, out):
    bbs, succ = blocks(body)
    state = {0: ((), (("exec", "full"),))} if bbs else {}
    work = [0] if bbs else []
    while work:
        i = work.pop()
        q, c = state[i][0], dict(state[i][1])
        for no, s, in_asm in bbs[i][1]:
            q = step(q, s, in_asm, lambda *a: None)
            c = consts_step(c, s)
        last = bbs[i][1][-1][1] if bbs[i][1] else ""
        fall = [j for j in succ[i] if j == i + 1]
        targets = [j for j in succ[i] if j != i + 1]
        for j in feasible_succ(c, last, targets, fall):
            cc = tuple(sorted(c.items()))
            if j in state:
                nq = join(state[j][0], q)
                nc = tuple(sorted(set(state[j][1]) & set(cc)))
            else:
                nq, nc = q, cc
            if state.get(j) != (nq, nc):
                state[j] = (nq, nc)
                work.append(j)
    bad = []
    for i, (label, insts) in enumerate(bbs):
        if i not in state:
            continue
        q = state[i][0]
        for no, s, in_asm in insts:
            q = step(q, s, in_asm, lambda s, hit, no=no: bad.append((no, s, sorted(hit))))
    for no, s, hit in bad:
        out.append(f"line {no}: {name}: `{s}` names in-flight v{hit}")
    return len(bad)


def check(path):
    lines = open(path).read().split("\n")
    out = []
    n = sum(check_kernel(name, body, out) for name, body in kernels(lines))
    for o in out:
        print(f"{path}:{o}")
    return n


if __name__ == "__main__":
    p = sys.argv[1] if len(sys.argv) > 1 else "build/asm/checksummer-gfx950.s"
    n = check(p)
    print(f"check_inflight: {n} hazard(s) in {p}")
    sys.exit(1 if n else 0)
