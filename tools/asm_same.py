#!/usr/bin/env python3
"""Are the product kernels' instruction streams the same as at another commit?

Builds the device assembly of xsknf_amd/csrc/checksummer.hip as it was at REV
(into a scratch directory) and compares it kernel by kernel with the current
product assembly (`make asm` -> build/asm/checksummer-gfx950.s), ignoring
labels, comments and directives.  Use it to tell whether profiles recorded at
REV still describe the product's kernels:

    python3 tools/asm_same.py <rev> [--diff]

--diff prints the instruction diff of every kernel that is not identical
(a renamed twin is matched by name with its template arguments removed).

    python3 tools/asm_same.py --ab

compares every product kernel with the kernel of the same name in the A/B build
(`make ab` -> build/ab/checksummer-gfx950.s): the A/B switches live in
checksummer_ab.h, and the shared kernels must be instruction-identical.
"""
import difflib
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-inline-asm", "-fvisibility=hidden", "--offload-arch=gfx950",
         "--cuda-device-only", "-S"]
FILES = ["xsknf_amd/csrc/checksummer.hip", "xsknf_amd/csrc/checksummer_internal.h", "include/xsknf_gpu.h"]


def kernels(path):
    out, cur = {}, None
    for line in open(path):
        m = re.match(r"^(_ZN9xsknf_gpu\w+):", line)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if cur is None:
            continue
        t = line.strip()
        if t.startswith(".Lfunc_end"):
            cur = None
            continue
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        out[cur].append(re.sub(r"\.LBB\d+_\d+", "L", t.split(";")[0].strip()))
    return out


def vs_ab():
    subprocess.run(["make", "-C", ROOT, "asm", "ab"], check=True, stdout=subprocess.DEVNULL)
    only_k = lambda d: {k: v for k, v in d.items() if "kernel" in k}   # (device globals match the pattern too)
    a = only_k(kernels(os.path.join(ROOT, "build", "asm", "checksummer-gfx950.s")))
    b = only_k(kernels(os.path.join(ROOT, "build", "ab", "checksummer-gfx950.s")))
    # the same instructions, scheduled or register-assigned differently
    regs = lambda ins: sorted(re.sub(r"\b([vs])(\d+)\b|\b([vs])\[\d+:\d+\]", r"\1\3#", x) for x in ins)
    same = [k for k in sorted(a) if k in b and a[k] == b[k]]
    renamed = [k for k in sorted(a) if k in b and a[k] != b[k] and regs(a[k]) == regs(b[k])]
    bad = [k for k in sorted(a) if k not in b or regs(a[k]) != regs(b[k])]
    for k in renamed:
        print(f"same instructions, scheduled / register-assigned differently: {k}")
    for k in bad:
        print(f"differs: {k}" if k in b else f"not in the A/B build: {k}")
    print(f"{len(same)} product kernels identical in the A/B build, {len(renamed)} the same instructions "
          f"scheduled or register-assigned differently, {len(bad)} not ({len(set(b) - set(a))} A/B-only kernels)")
    return 0 if not bad else 1


def main():
    if sys.argv[1:] == ["--ab"]:
        return vs_ab()
    args = [a for a in sys.argv[1:] if a != "--diff"]
    show = "--diff" in sys.argv[1:]
    if len(args) != 1:
        raise SystemExit(__doc__)
    rev = args[0]
    cur = os.path.join(ROOT, "build", "asm", "checksummer-gfx950.s")
    subprocess.run(["make", "-C", ROOT, "asm"], check=True, stdout=subprocess.DEVNULL)
    with tempfile.TemporaryDirectory() as d:
        for f in FILES:
            os.makedirs(os.path.join(d, os.path.dirname(f)), exist_ok=True)
            with open(os.path.join(d, f), "wb") as fh:
                fh.write(subprocess.run(["git", "-C", ROOT, "show", f"{rev}:{f}"], check=True,
                                        stdout=subprocess.PIPE).stdout)
        old = os.path.join(d, "old.s")
        subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, "-Iinclude", "-o", old, FILES[0]], cwd=d, check=True)
        a, b = kernels(old), kernels(cur)
    same, bad = 0, 0
    for k in sorted(set(a) & set(b)):
        if a[k] == b[k]:
            same += 1
        else:
            bad += 1
            print(f"differs: {k} ({len(a[k])} vs {len(b[k])} instructions)")
    # a kernel renamed (a template parameter added) with the same instructions
    gone, new = sorted(set(a) - set(b)), sorted(set(b) - set(a))
    for k in gone:
        twin = next((j for j in new if b[j] == a[k]), None)
        if twin:
            new.remove(twin)
            same += 1
            print(f"renamed, identical: {k} -> {twin}")
        else:
            bad += 1
            print(f"only at {rev}: {k}")
    for j in new:
        bad += 1
        print(f"only now: {j}")
    if show:
        # differing kernels, and kernels present on one side only paired by family name
        fam = lambda k: re.sub(r"I.*E(EvNS|vNS)", "", k)
        pairs = [(k, k) for k in sorted(set(a) & set(b)) if a[k] != b[k]]
        pairs += [(k, j) for k in gone for j in new if fam(k) == fam(j) and
                  len(set(a[k]) ^ set(b[j])) < 200]
        for k, j in pairs:
            print(f"--- {k} ({rev})\n+++ {j} (now)")
            for line in difflib.unified_diff(a[k], b[j], lineterm="", n=0):
                if not line.startswith(("---", "+++")):
                    print(line)
    print(f"{same} kernels identical to {rev}, {bad} not")
    return 0 if bad == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
