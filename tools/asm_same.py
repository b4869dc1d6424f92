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


def main():
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
