"""Golden fixtures (tests/golden/): the oracle reproduces them on CPU, the
gfx950 path (through the C ABI) reproduces them on the GPU, and the known-answer
table matches the KATs the oracle tests use."""
import json
import os

import numpy as np
import pytest

from oracle import csum_oracle as O
from xsknf_amd import frames

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = np.load(os.path.join(HERE, "golden", "checksummer_golden.npz"))
NAMES = sorted({k.split("__")[0] for k in GOLD.files} - {"meta"})


def case(name):
    umem = GOLD[f"{name}__umem"].copy()
    descs = GOLD[f"{name}__descs"].copy().view(frames.DESC_DTYPE).reshape(-1)
    it, act, nif, ing = (int(x) for x in GOLD[f"{name}__opts"])
    expected = umem.copy()
    expected[GOLD[f"{name}__pos"]] = GOLD[f"{name}__val"]
    return umem, descs, dict(iters=it, action=act, nif=nif, ingress=ing), GOLD[f"{name}__verdicts"], expected


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_golden(name):
    umem, descs, kw, v_exp, u_exp = case(name)
    v = O.c_process_batch(umem, descs, **kw)
    assert np.array_equal(v, v_exp)
    assert np.array_equal(umem, u_exp)


def test_known_answer_table_matches_oracle_tests():
    from tests.test_oracle import KATS
    table = {c["id"]: c for c in json.load(open(os.path.join(HERE, "golden", "known_answers.json")))["cases"]}
    for name, frame, kw, ret, sl, chk in KATS:
        key = {"C6-tcp": "C6a", "C6-33": "C6b", "C6-13": "C6c", "C6-ihl15": "C6d", "C6-ihl6": "C6e"}.get(name, name)
        assert table[key]["ret"] == ret
        if chk is not None:
            assert table[key]["check"] == chk and table[key]["check_at"] == sl[0]


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_reproduces_golden(name):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from xsknf_amd import Checksummer, ChecksummerOptions
    umem, descs, kw, v_exp, u_exp = case(name)
    cs = Checksummer(ChecksummerOptions(action=kw["action"], csum_iterations=kw["iters"]),
                     num_interfaces=kw["nif"], frame_len_hint=int(descs["len"].max()))
    du = torch.from_numpy(umem).cuda()
    dd = torch.from_numpy(descs.view(np.uint8).reshape(-1, 16).copy()).cuda()
    v = cs.process_batch(du, dd, ingress_ifindex=kw["ingress"])
    torch.cuda.synchronize()
    assert np.array_equal(v.cpu().numpy(), v_exp)
    assert np.array_equal(du.cpu().numpy(), u_exp)
