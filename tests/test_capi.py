"""The C-ABI library: builds for gfx950, loads without a GPU, and exports every
function include/*.h declares.  Argument validation paths that return before
any HIP call are exercised here too (no compute calls without a GPU)."""
import ctypes
import errno
import glob
import os
import re
import subprocess

import pytest

from xsknf_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions(header="xsknf_gpu.h", api="XSKNF_GPU_API"):
    """Functions a header declares with its export macro (include/xsknf_gpu.h:
    XSKNF_GPU_API -> libxsknf_gpu.so; include/xsknf.h: XSKNF_API -> libxsknf.so)."""
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set()
    for m in re.finditer(rf"\b{api}\b[^;(]*?\b(xsknf_\w+)\s*\(", src):
        names.add(m.group(1))
    return sorted(names)


def test_every_header_is_covered():
    assert sorted(os.path.basename(h) for h in glob.glob(os.path.join(ROOT, "include", "*.h"))) == \
        ["xsknf.h", "xsknf_gpu.h"]


def test_header_declares_the_binding_list():
    assert set(declared_functions()) == set(_lib.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    for name in declared_functions():
        assert re.search(rf"\bT {name}\b", out), f"{name} not exported as a text symbol"


def test_library_has_gfx950_code_object():
    blob = open(_lib.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"hipv4-amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}, targets


def test_version():
    assert _lib.load().xsknf_gpu_version() == 1


def test_argument_validation_without_gpu():
    lib = _lib.load()
    f = lib.xsknf_gpu_checksum_batch
    good = _lib.CsumOpts(1, _lib.ACTION_REDIRECT, 1, 0)
    # n == 0 is a no-op
    assert f(None, 0, None, 0, 0, ctypes.byref(good), None, 0, None) == 0
    # NULL opts, bad action, REDIRECT with 0 interfaces, reserved != 0
    assert f(None, 0, None, 0, 0, None, None, 0, None) == -errno.EINVAL
    for bad in (_lib.CsumOpts(1, 2, 1, 0), _lib.CsumOpts(1, _lib.ACTION_REDIRECT, 0, 0),
                _lib.CsumOpts(1, _lib.ACTION_DROP, 1, 7)):
        assert f(None, 0, None, 5, 0, ctypes.byref(bad), None, 0, None) == -errno.EINVAL
    # DROP does not need interfaces (the reference never divides in DROP mode)
    assert f(None, 0, None, 0, 0, ctypes.byref(_lib.CsumOpts(1, _lib.ACTION_DROP, 0, 0)),
             None, 0, None) == 0
    # NULL buffers with n > 0
    assert f(None, 0, None, 5, 0, ctypes.byref(good), None, 0, None) == -errno.EINVAL


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(_lib.XsknfGpuError):
        _lib.load()


def test_only_declared_symbols_are_exported():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    assert exported == set(declared_functions())


def test_ctx_argument_validation_without_gpu():
    lib = _lib.load()
    ctx = ctypes.c_void_p()
    assert lib.xsknf_gpu_ctx_create(None, 0, 0, 16, 0) == -errno.EINVAL
    assert lib.xsknf_gpu_ctx_create(ctypes.byref(ctx), 0, 7, 16, 0) == -errno.EINVAL
    assert lib.xsknf_gpu_ctx_create(ctypes.byref(ctx), 0, 0, 0, 0) == -errno.EINVAL
    assert lib.xsknf_gpu_ctx_process_batch(None, None, 0, 0, None, None) == -errno.EINVAL
    assert lib.xsknf_gpu_ctx_destroy(None) == -errno.EINVAL


def test_launch_shape_for_lengths_without_gpu():
    """xsknf_gpu_launch_cfg_for_lens: the largest frame picks the kernel family
    and the header window; for <= 4 KiB frames the mean picks the CU-wide tile
    pool (window + 32; also for an unknown mean) or, for a mix of mostly short
    frames (mean < 512), 4-wave blocks with the static schedule."""
    lib = _lib.load()

    def shape(mx, mean):
        c = _lib.LaunchCfg()
        assert lib.xsknf_gpu_launch_cfg_for_lens(mx, mean, ctypes.byref(c)) == 0
        return c.kernel, c.lanes_per_frame, c.chunks_per_lane, c.window_chunks, c.fused_stores

    plain = _lib.LaunchCfg()
    assert lib.xsknf_gpu_default_launch_cfg(1500, ctypes.byref(plain)) == 0
    for mean in (0, 512, 1023, 1500):
        assert shape(1500, mean) == (plain.kernel, plain.lanes_per_frame, plain.chunks_per_lane,
                                     plain.window_chunks, plain.fused_stores)
    assert shape(1500, 1500)[2] == 2 and shape(1500, 1500)[3] == 56
    assert shape(1500, 352)[3] == 24 and shape(1500, 511)[3] == 24 and shape(4000, 1024)[3] == 56
    assert shape(9000, 9000)[3] == 52          # jumbo: 4-chunk window, tile pool, whatever the mean
    assert shape(64, 64)[1] == 1               # lane kernel
    assert shape(64, 64)[3] == 1024            # windows transposed where a tile's frames lie apart
    assert lib.xsknf_gpu_launch_cfg_for_lens(1500, 1500, None) == -errno.EINVAL


def test_one_hip_runtime_per_process():
    """Loading the library before torch must not leave two HIP runtimes in the
    process (ROCm's and torch's bundled one): _lib.load() binds to torch's."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from xsknf_amd import _lib; _lib.load()\n"
            "import torch\n"
            "maps = open('/proc/self/maps').read().split('\\n')\n"
            "hip = sorted({l.split()[-1] for l in maps if 'libamdhip64' in l})\n"
            "hsa = sorted({l.split()[-1] for l in maps if 'libhsa-runtime64' in l})\n"
            "print(len(hip), len(hsa))\n") % ROOT
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.split() == ["1", "1"], out.stdout
