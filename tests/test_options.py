"""Host-side mirrors of the reference's option parsing: checksummer_user.c:139-175
(app options, getopt "qxai:c:") and src/xsknf.c:777-874 (library options)."""
import pytest

from xsknf_amd import ACTION_DROP, ACTION_REDIRECT, parse_args, parse_command_line


def test_app_defaults_match_reference_globals():
    o = parse_command_line([])
    assert o.action == ACTION_REDIRECT and o.csum_iterations == 1      # :24-25
    assert not (o.quiet or o.extra_stats or o.app_stats)


def test_app_options_as_the_harness_passes_them():
    # tests/test-drop-cpu.py:80 runs `... -- -q -i <iter> -c DROP`
    o = parse_command_line(["-q", "-i", "7", "-c", "DROP"])
    assert o.quiet and o.csum_iterations == 7 and o.action == ACTION_DROP
    o = parse_command_line(["-x", "-a", "-c", "REDIRECT", "-i", "-2"])
    assert o.extra_stats and o.app_stats and o.action == ACTION_REDIRECT and o.csum_iterations == -2


def test_atoi_semantics_of_csum_iterations():
    assert parse_command_line(["-i", "12abc"]).csum_iterations == 12
    assert parse_command_line(["-i", "abc"]).csum_iterations == 0


def test_invalid_action_exits_with_usage(capsys):
    with pytest.raises(SystemExit) as e:
        parse_command_line(["-c", "FORWARD"])
    assert e.value.code == 1
    err = capsys.readouterr().err
    assert "ERROR: invalid action FORWARD" in err and "Usage:" in err


def test_library_options_and_defaults():
    cfg, app = parse_args(["-i", "veth1b:c", "-S", "--", "-q", "-c", "DROP"])
    assert cfg.interfaces == ["veth1b"] and cfg.bind_flags == ["copy"] and cfg.skb_mode
    assert cfg.batch_size == 64 and cfg.workers == 1 and cfg.xsk_frame_size == 4096   # :46-52
    assert app == ["-q", "-c", "DROP"]
    cfg, _ = parse_args(["-i", "eth0:z", "-i", "eth1", "-b", "256", "-B", "-w", "4", "-u", "-f", "9000",
                         "-M", "COMBINED", "-p"])
    assert cfg.num_interfaces == 2 and cfg.bind_flags == ["zerocopy", ""]
    assert cfg.batch_size == 256 and cfg.busy_poll and cfg.workers == 4 and cfg.poll
    assert cfg.unaligned_chunks and cfg.xsk_frame_size == 9000 and cfg.working_mode == 3


@pytest.mark.parametrize("argv", [
    [],                                   # no interface (:857-860)
    ["-i", "eth0:q"],                     # unknown copy mode (:801-805)
    ["-i", "eth0", "-M", "FAST"],         # unknown mode (:841-843)
    ["-i", "eth0", "-w", "0"],            # workers < 1 (:846-850)
    ["-i", "eth0", "-f", "3000"],         # non-power-of-two frame size, aligned (:866-871)
])
def test_library_option_errors_exit_1(argv):
    with pytest.raises(SystemExit) as e:
        parse_args(argv)
    assert e.value.code == 1
