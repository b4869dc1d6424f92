"""tools/check_inflight.py: the build-time guard of the split kernel's inline-asm
load pipeline (a register of an outstanding asm load named before its wait)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import check_inflight as C  # noqa: E402

HEAD = "_Zkern:\n"
TAIL = "\ts_endpgm\n.Lfunc_end0:\n"


def load(dst, addr):
    return f"\t;;#ASMSTART\n\tglobal_load_dwordx4 {dst}, {addr}, off nt\n\t;;#ASMEND\n"


def wait(n):
    return f"\t;;#ASMSTART\n\ts_waitcnt vmcnt({n})\n\t;;#ASMEND\n"


def hazards(text, tmp_path):
    p = tmp_path / "k.s"
    p.write_text(HEAD + text + TAIL)
    return C.check(str(p))


def test_copy_before_wait_is_reported(tmp_path):
    body = load("v[20:23]", "v[16:17]") + "\tv_mov_b64_e32 v[46:47], v[22:23]\n" + wait(0)
    assert hazards(body, tmp_path) == 1


def test_use_after_counted_wait_is_clean(tmp_path):
    body = (load("v[20:23]", "v[16:17]") + load("v[24:27]", "v[18:19]") + wait(1) +
            "\tv_mov_b32_e32 v40, v20\n" + wait(0) + "\tv_mov_b32_e32 v41, v24\n")
    assert hazards(body, tmp_path) == 0


def test_wait_counts_only_older_loads(tmp_path):
    # vmcnt(1) leaves the younger load outstanding: naming it is a hazard
    body = load("v[20:23]", "v[16:17]") + load("v[24:27]", "v[18:19]") + wait(1) + "\tv_mov_b32_e32 v41, v25\n"
    assert hazards(body, tmp_path) == 1


def test_loop_back_edge_carries_outstanding_loads(tmp_path):
    # a load issued at the bottom of a loop is outstanding at its top
    body = (".LBB0_1:\n\tv_add_u32_e32 v21, 1, v2\n" + load("v[20:23]", "v[16:17]") +
            "\ts_cmp_lg_u32 s0, 0\n\ts_cbranch_scc1 .LBB0_1\n" + wait(0))
    # the add writes into the outstanding load, and so does the reissued load
    assert hazards(body, tmp_path) == 2


def test_skip_edge_of_a_partial_exec_is_followed(tmp_path):
    # the wait sits in an exec-masked region: the skip edge bypasses it
    body = (load("v[20:23]", "v[16:17]") + "\ts_and_saveexec_b64 s[0:1], vcc\n\ts_cbranch_execz .LBB0_2\n" +
            wait(0) + ".LBB0_2:\n\ts_or_b64 exec, exec, s[0:1]\n\tv_mov_b32_e32 v40, v20\n")
    assert hazards(body, tmp_path) == 1
