"""The gfx950 path against the REFERENCE's own function, directly.

`oracle/_ref/libcsum_ref.so` is checksummer_user.c:30-112 compiled from its
verbatim lines (oracle/ref.py; built in the build container, it travels to the
GPU box as a built library -- the reference checkout itself is never read
here).  The other GPU tests compare with the restatement, which
tests/test_ref_pin.py pins to this library on CPU; these compare the HIP path
with the library itself, through the C ABI, on seeded randomized batches that
cover every branch of :34-55, odd starts, iterations -3..7919, both actions,
1-4 interfaces, every launch family (lane kernel, split kernel with and
without the pool, jumbo) and the three host paths.  Bit-exact: every verdict
and every UMEM byte.  A GPU run without the library fails (it is not skipped).
"""
import numpy as np
import pytest

from oracle import ref as R
from xsknf_amd import Checksummer, ChecksummerOptions, frames

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not R.available():   # required on a GPU box (tests/oracles.py): no skip
        pytest.fail(f"{R.LIB_PATH} not built: run build() where the reference checkout exists")
    return torch.device("cuda:0")


def _batch(seed, n, max_len, layout):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, max_len + 1, size=n).astype(np.uint32)
    lens[: n // 10] = rng.integers(0, 64, size=n // 10)
    if layout == "aligned":
        lens = np.minimum(lens, 2048 - 256)
        b = frames.aligned_batch(n, lens, seed=seed)
    else:
        b = frames.unaligned_batch(n, lens, seed=seed)
    frames.inject_edge_cases(b, 0.3, seed=seed + 1)
    offs = b.frame_offsets()
    for i in rng.choice(n, size=n // 8, replace=False):   # every ihl nibble on well-formed frames
        if b.descs["len"][i] >= 15:
            b.umem[int(offs[i]) + 14] = (b.umem[int(offs[i]) + 14] & 0xF0) | int(rng.integers(0, 16))
    return b


CASES = [
    # (seed, frames, longest frame, layout, hint, iterations, action, interfaces, ingress)
    (1, 3000, 128, "aligned", 64, 1, 0, 1, 0),          # lane kernel
    (2, 3000, 128, "unaligned", 100, 3, 1, 1, 0),
    (3, 5000, 1792, "aligned", 1500, 1, 0, 2, 1),       # split kernel, pool
    (4, 5000, 1600, "unaligned", 1500, -3, 0, 3, 2),
    (5, 800, 9100, "unaligned", 9000, 2, 0, 4, 3),      # jumbo shape
    (6, 1000, 300, "aligned", 300, 7919, 1, 1, 0),      # u32 wrap of the repeated sum
    (7, 6000, 1500, "aligned", 0, 0, 0, 1, 0),          # no payload sum
    (8, 20000, 1500, "unaligned", 1500, 5, 0, 2, 0),
]


@pytest.mark.parametrize("case", CASES, ids=[f"seed{c[0]}" for c in CASES])
def test_device_batches_equal_the_reference(dev, case):
    seed, n, max_len, layout, hint, it, act, nif, ing = case
    b = _batch(seed, n, max_len, layout)
    ref = b.copy()
    rv = R.process_batch(ref.umem, ref.descs, ingress=ing, iters=it, action=act, nif=nif)
    cs = Checksummer(ChecksummerOptions(action=act, csum_iterations=it), num_interfaces=nif, frame_len_hint=hint)
    umem = torch.from_numpy(b.umem).to(dev)
    descs = torch.from_numpy(b.descs.view(np.uint8).reshape(-1, 16).copy()).to(dev)
    v = cs.process_batch(umem, descs, ingress_ifindex=ing)
    torch.cuda.synchronize()
    gv, gu = v.cpu().numpy(), umem.cpu().numpy()
    bad = np.nonzero(gv != rv)[0]
    assert bad.size == 0, f"verdicts differ at {bad[:8]}: gpu {gv[bad[:8]]} reference {rv[bad[:8]]}"
    diff = np.nonzero(gu != ref.umem)[0]
    assert diff.size == 0, f"{diff.size} UMEM bytes differ, first at {diff[:8]}"


@pytest.mark.parametrize("path", ["zerocopy", "staged", "resident"])
def test_host_paths_equal_the_reference(dev, path):
    from xsknf_amd import HostPath
    b = _batch(99, 4000, 1600, "unaligned")
    ref = b.copy()
    rv = R.process_batch(ref.umem, ref.descs, ingress=1, iters=2, action=0, nif=3)
    cs = Checksummer(ChecksummerOptions(action=0, csum_iterations=2), num_interfaces=3, frame_len_hint=1500)
    umem = b.umem.copy()
    with HostPath(cs, umem, path=path, max_batch=4096) as hp:
        v = np.concatenate([hp.process_batch(b.descs[lo:lo + 500], ingress_ifindex=1) for lo in range(0, b.n, 500)])
    assert np.array_equal(v, rv)
    assert np.array_equal(umem, ref.umem)


@pytest.mark.parametrize("seed", range(24))
def test_random_sweep_equals_the_reference(dev, seed):
    """Randomized cases against the reference's function, one per seed: frame
    count, longest frame (0 .. 9100 B: every launch family the hint picks),
    layout, the hint given (right, 0 = unknown, or too small: a hint is only a
    hint), the mean given or not, iterations -3 .. 7919, action, 1-4
    interfaces, ingress, and half of the batches with NIC-offloaded checks (the
    kernels' write elision) before the edge cases."""
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.integers(1, 6000))
    max_len = int(rng.choice([64, 128, 200, 600, 1500, 1792, 4000, 9100]))
    layout = "aligned" if max_len <= 1792 and rng.random() < 0.5 else "unaligned"
    lens = rng.integers(0, max_len + 1, size=n).astype(np.uint32)
    if layout == "aligned":
        b = frames.aligned_batch(n, lens, seed=seed)
    else:
        b = frames.unaligned_batch(n, lens, seed=seed)
    if rng.random() < 0.5:
        frames.offload_checks_host(b)
    frames.inject_edge_cases(b, float(rng.uniform(0.02, 0.3)), seed=seed + 7)
    it = int(rng.choice([-3, 0, 1, 2, 3, 5, 17, 255, 7919]))
    act, nif, ing = int(rng.integers(0, 2)), int(rng.integers(1, 5)), int(rng.integers(0, 6))
    hint = int(rng.choice([0, max_len, max(1, max_len // 3)]))
    mean = int(b.descs["len"].mean()) if rng.random() < 0.5 else 0
    ref = b.copy()
    rv = R.process_batch(ref.umem, ref.descs, ingress=ing, iters=it, action=act, nif=nif)
    cs = Checksummer(ChecksummerOptions(action=act, csum_iterations=it), num_interfaces=nif,
                     frame_len_hint=hint, frame_len_mean=mean)
    umem = torch.from_numpy(b.umem).to(dev)
    descs = torch.from_numpy(b.descs.view(np.uint8).reshape(-1, 16).copy()).to(dev)
    v = cs.process_batch(umem, descs, ingress_ifindex=ing)
    torch.cuda.synchronize()
    gv, gu = v.cpu().numpy(), umem.cpu().numpy()
    bad = np.nonzero(gv != rv)[0]
    assert bad.size == 0, f"verdicts differ at {bad[:8]}: gpu {gv[bad[:8]]} reference {rv[bad[:8]]}"
    diff = np.nonzero(gu != ref.umem)[0]
    assert diff.size == 0, f"{diff.size} UMEM bytes differ, first at {diff[:8]}"
