"""The AF_XDP worker loop with the GPU batch hook (libxsknf_gpu's
xsknf_gpu_hook_process) as the NF: every rx batch the runtime peeks is
checksummed by one gfx950 launch on the worker's host UMEM, then routed by the
returned verdicts (src/xsknf.c:654-714 with the per-frame loop replaced).

Emulated queues play the kernel's part (the GPU box runs unprivileged, so
there are no AF_XDP sockets there); results must equal the oracle applied per
frame, byte for byte and in order.
"""
import pytest

from oracle import csum_oracle as O
from xsknf_amd import _lib
from xsknf_amd import runtime as R

from test_runtime import config1, expected, pump

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def frames():
    return config1.frames_check(9000)


def run_loop(cfg, plan, n_if=1, two_phase=False, depth=1, **hook_kw):
    hook = R.GpuHook(workers=cfg.workers, max_batch=cfg.batch_size, num_interfaces=n_if,
                     frame_len_hint=cfg.xsk_frame_size, **hook_kw)
    rt = R.Runtime(cfg)
    try:
        if two_phase:   # xsknf_gpu_hook_submit / _complete: one batch in flight per worker
            rt.set_batch_processor_async(hook.submit_ptr, hook.complete_ptr, hook.handle)
            rt.set_batch_depth(depth)
        else:
            rt.set_batch_processor(hook.fn_ptr, hook.handle)
        rt.start()
        got = pump(rt, plan, n_if=n_if, timeout=60)
        assert rt.stop() == 0
        hs = hook.stats(0)
        st = [rt.stats(0, i) for i in range(n_if)]
    finally:
        rt.stop()
        hook.destroy()
        rt.close()
    return got, hs, st


@pytest.mark.parametrize("two_phase", [False, True], ids=["one-call", "two-phase"])
@pytest.mark.parametrize("path", [_lib.PATH_ZEROCOPY, _lib.PATH_STAGED], ids=["zerocopy", "staged"])
@pytest.mark.parametrize("batch", [64, 2048])
def test_gpu_hook_redirect_matches_oracle(frames, path, batch, two_phase):
    cfg = R.make_config(["emu0"], batch_size=batch)
    got, hs, st = run_loop(cfg, {0: frames}, two_phase=two_phase, path=path, iterations=2)
    want = [b for v, b in expected(frames, iterations=2) if v != -1]
    assert got[0] == want
    assert hs["frames"] == len(frames) == st[0]["rx_npkts"]
    assert hs["batches"] >= len(frames) // batch


@pytest.mark.parametrize("path", [_lib.PATH_ZEROCOPY, _lib.PATH_STAGED, _lib.PATH_RESIDENT],
                         ids=["zerocopy", "staged", "resident"])
@pytest.mark.parametrize("depth", [2, 4, 8])
def test_gpu_hook_batches_in_flight(frames, path, depth):
    """Two-phase hook with up to `depth` batches out per worker (a launched
    context has 5 slots: past 4 out its submit waits for its oldest piece; the
    resident ring has 8 entries)."""
    cfg = R.make_config(["emu0"], batch_size=64)
    got, hs, st = run_loop(cfg, {0: frames}, two_phase=True, depth=depth, path=path, iterations=3)
    assert got[0] == [b for v, b in expected(frames, iterations=3) if v != -1]
    assert hs["frames"] == len(frames) == st[0]["rx_npkts"]


def test_gpu_hook_drop(frames):
    cfg = R.make_config(["emu0"], batch_size=512)
    got, hs, st = run_loop(cfg, {0: frames}, action=_lib.ACTION_DROP)
    assert got[0] == [b for v, b in expected(frames, action=O.DROP) if v != -1]
    assert st[0]["rx_npkts"] == len(frames)


def test_gpu_hook_unaligned(frames):
    cfg = R.make_config(["emu0"], batch_size=1024, unaligned=True, frame_size=3000)
    got, _, _ = run_loop(cfg, {0: frames[:6000]}, iterations=5)
    assert got[0] == [b for v, b in expected(frames[:6000], iterations=5) if v != -1]


@pytest.mark.parametrize("two_phase", [False, True], ids=["one-call", "two-phase"])
@pytest.mark.parametrize("bind", [(0, 0), (R.XDP_COPY, R.XDP_ZEROCOPY)], ids=["shared-umem", "two-umems"])
def test_gpu_hook_two_interfaces(frames, bind, two_phase):
    f0, f1 = frames[:4000], frames[4000:8000]
    cfg = R.make_config(["emu0", "emu1"], batch_size=256, bind=list(bind))
    got, _, _ = run_loop(cfg, {0: f0, 1: f1}, n_if=2, two_phase=two_phase)
    e0, e1 = expected(f0, 0, nif=2), expected(f1, 1, nif=2)
    assert sorted(got[0]) == sorted([b for v, b in e0 + e1 if v == 0])
    assert sorted(got[1]) == sorted([b for v, b in e0 + e1 if v == 1])
