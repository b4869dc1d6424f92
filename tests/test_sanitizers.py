"""The host runtime (libxsknf's C sources) and the CPU oracle under
ThreadSanitizer and AddressSanitizer + UBSan: two worker
threads, two emulated interfaces, REDIRECT and DROP, the per-frame NF and the
two-phase batch hook, checked frame by frame against the oracle
(tests/c/san_runtime.c).  CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = ["tests/c/san_runtime.c", "xsknf_amd/csrc/xsknf_rt.c", "xsknf_amd/csrc/rt_netlink.c",
        "oracle/csum_oracle.c"]


@pytest.fixture(scope="module")
def builds(tmp_path_factory):
    if not shutil.which("gcc"):
        pytest.skip("gcc missing")
    d = tmp_path_factory.mktemp("san")
    out = {}
    for name, flags in (("tsan", ["-fsanitize=thread"]), ("asan", ["-fsanitize=address,undefined",
                                                                    "-fno-sanitize-recover=undefined"])):
        exe = str(d / name)
        subprocess.run(["gcc", "-O1", "-g", "-std=gnu11", "-fno-omit-frame-pointer", *flags, "-Iinclude",
                        *SRCS, "-pthread", "-lm", "-o", exe], cwd=ROOT, check=True)
        out[name] = exe
    return out


@pytest.mark.parametrize("san", ["tsan", "asan"])
@pytest.mark.parametrize("action", ["redirect", "drop"])
@pytest.mark.parametrize("hook", ["per-frame", "async"])
def test_runtime_is_sanitizer_clean(builds, san, action, hook):
    """hook "async": the two-phase batch hook (one batch in flight per worker)."""
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1")
    r = subprocess.run([builds[san], action, hook], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    assert "bad 0" in r.stdout


def test_shard_arithmetic_is_sanitizer_clean(tmp_path):
    """The multi-device path's host arithmetic (xsknf_amd/csrc/shard_plan.cpp:
    shard cuts, span rebasing, the packed layout) under AddressSanitizer + UBSan
    on 3000 random and edge-case descriptor sets (tests/c/san_shard.c), with its
    invariants checked."""
    if not shutil.which("g++"):
        pytest.skip("g++ missing")
    exe = str(tmp_path / "san_shard")
    subprocess.run(["g++", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=undefined", "-Iinclude", "-x", "c", "tests/c/san_shard.c", "-x", "c++",
                    "-std=c++17", "xsknf_amd/csrc/shard_plan.cpp", "-o", exe], cwd=ROOT, check=True)
    r = subprocess.run([exe], cwd=ROOT, env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"), capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    assert r.stdout.strip() == "ok 3000"
