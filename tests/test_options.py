"""The reference's option parsing: checksummer_user.c:139-175 (app options,
getopt "qxai:c:", mirrored for the Python API) and src/xsknf.c:777-874 (library
options: the runtime's C xsknf_parse_args, bound by runtime.parse_args -- one
parser for the binary and the Python API)."""
import pytest

from xsknf_amd import ACTION_DROP, ACTION_REDIRECT, parse_command_line
from xsknf_amd import runtime as R


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
    assert "action 'FORWARD' is neither REDIRECT nor DROP" in err and "usage:" in err


def test_library_options_and_defaults():
    cfg, app = R.parse_args(["-i", "veth1b:c", "-S", "--", "-q", "-c", "DROP"])
    assert cfg.num_interfaces == 1 and cfg.interfaces[0] == b"veth1b"
    assert cfg.bind_flags[0] == R.XDP_USE_NEED_WAKEUP | R.XDP_COPY
    assert cfg.xdp_flags & R.XDP_FLAGS_SKB_MODE and not cfg.xdp_flags & R.XDP_FLAGS_DRV_MODE
    assert cfg.batch_size == 64 and cfg.workers == 1 and cfg.xsk_frame_size == 4096   # :46-52
    assert cfg.working_mode == R.MODE_AF_XDP
    assert app == ["-q", "-c", "DROP"]
    cfg, app = R.parse_args(["-i", "eth0:z", "-i", "eth1", "-b", "256", "-B", "-w", "4", "-u", "-f", "9000",
                             "-M", "COMBINED", "-p"])
    assert cfg.num_interfaces == 2 and [cfg.interfaces[i] for i in range(2)] == [b"eth0", b"eth1"]
    assert cfg.bind_flags[0] == R.XDP_USE_NEED_WAKEUP | R.XDP_ZEROCOPY and cfg.bind_flags[1] == R.XDP_USE_NEED_WAKEUP
    assert cfg.batch_size == 256 and cfg.busy_poll and cfg.workers == 4 and cfg.poll
    assert cfg.unaligned_chunks and cfg.xsk_frame_size == 9000 and cfg.working_mode == R.MODE_COMBINED
    assert cfg.xdp_flags & R.XDP_FLAGS_DRV_MODE and app == []
    # the app's own parser takes what follows `--`, as checksummer_user.c:197 resumes getopt there
    cfg, app = R.parse_args(["--iface=ens1f0", "--", "-i", "5", "-c", "DROP"])
    o = parse_command_line(app)
    assert cfg.interfaces[0] == b"ens1f0" and o.csum_iterations == 5 and o.action == ACTION_DROP


@pytest.mark.parametrize("argv,msg", [
    (["-i", "eth0:q"], "copy mode 'q' is neither c nor z"),              # src/xsknf.c:800-812
    (["-i", "eth0", "-M", "TURBO"], "no working mode named 'TURBO'"),     # :845-858
    (["-i", "eth0", "-w", "0"], "worker count '0' is not a positive number"),   # :859-866
    ([], "no interface given"),                                           # :872-874
    (["-i", "eth0", "-f", "3000"], "frame size 3000 must be a power of two"),   # :866-871
    (["-i", "eth0", "-Z"], "invalid option -- 'Z'"),                      # getopt, then the summary
])
def test_library_option_errors_exit_1_with_usage(argv, msg):
    """xsknf_parse_args ends the process on a bad library option, as the
    reference's does (usage() + exit(1)); runtime.parse_args therefore runs it
    in a child process here and checks the exit status and the message."""
    import subprocess
    import sys
    root = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from xsknf_amd import runtime as R\n"
            "R.parse_args(%r)\n"
            "print('returned')\n") % (root, argv)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 1, (p.returncode, p.stdout, p.stderr)
    assert msg in p.stderr and "returned" not in p.stdout
    assert "xsknf library options" in p.stderr and "--iface=IF" in p.stderr   # the option summary
