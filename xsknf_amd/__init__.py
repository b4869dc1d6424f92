"""xsknf_amd -- MI355X-native batch path for the xsknf checksummer NF.

The reference (FedeParola/xsknf) calls `xsknf_packet_processor()` once per
AF_XDP frame; here a whole rx batch is checksummed by one gfx950 kernel
(`xsknf_amd/csrc/checksummer.hip`) behind the C ABI of `include/xsknf_gpu.h`.
"""
from .checksummer import (ACTION_DROP, ACTION_REDIRECT, Checksummer, ChecksummerOptions, HostPath,
                          parse_command_line)
# The library options (src/xsknf.c:777-874) are parsed by the runtime's C
# xsknf_parse_args since round 2; these names keep the round-1 Python API
# importable (XsknfConfig is the ctypes struct xsknf_config).
from .runtime import Config as XsknfConfig
from .runtime import parse_args

__all__ = ["ACTION_DROP", "ACTION_REDIRECT", "Checksummer", "ChecksummerOptions", "HostPath",
           "XsknfConfig", "parse_args", "parse_command_line"]
__version__ = "0.1.0"
