"""bench.py's measurement bookkeeping, on CPU (no GPU calls): the rotation that
keeps a pass out of the Infinity Cache, the iteration schedule that makes every
step rewrite every check of a base workload, the stream / batch pairing of
--streams, and the NIC workloads' shapes."""
import numpy as np
import pytest

pytest.importorskip("torch")
import bench  # noqa: E402


class Args:
    rotate = 0
    rotate_bytes = 1 << 30
    streams = 1


def test_rotation_keeps_a_pass_past_the_infinity_cache():
    a = Args()
    assert bench.rotation(np.full(1 << 20, 1500, np.uint32), a) == 1
    k = bench.rotation(np.full(1 << 20, 64, np.uint32), a)
    touched = (1 << 20) * (64 + 20)
    assert k * touched >= a.rotate_bytes and (k - 1) * touched < a.rotate_bytes


@pytest.mark.parametrize("K", [1, 2, 3, 13])
def test_every_visit_of_a_batch_changes_its_checks(K):
    """Consecutive visits of the same batch use different iteration counts."""
    last = {}
    for it in range(10 * K):
        j, i = it % K, bench.iterations_of_step(it, K)
        if j in last:
            assert i != last[j]
        last[j] = i


@pytest.mark.parametrize("streams,lens,want", [(1, 64, (13, 1)), (2, 64, (14, 2)), (2, 1500, (2, 2)),
                                               (3, 1500, (3, 3))])
def test_batches_and_streams(streams, lens, want):
    a = Args()
    a.streams = streams
    K, S = bench.batches_and_streams("1500", np.full(1 << 20, lens, np.uint32), a)
    assert (K, S) == want
    assert K % S == 0                       # every visit of batch j goes to stream j % S
    for it in range(5 * K):
        assert (it % S) == (it % K) % S


def test_nic_workloads_time_one_stream_and_mirror_their_base():
    a = Args()
    a.streams = 2
    assert bench.batches_and_streams("1500-nic", np.full(16, 1500, np.uint32), a)[1] == 1
    for nic, base in bench.NIC.items():
        assert bench.WORKLOADS[nic][:3] == bench.WORKLOADS[base][:3]
