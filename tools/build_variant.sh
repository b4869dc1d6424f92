#!/bin/bash
# Build an A/B variant of the product library with extra -D flags (on the CPU
# container, before a gpurun call; the GPU box only loads the result):
#   tools/build_variant.sh <name> [-DXSKNF_...=N ...]   -> build/<name>/libxsknf_gpu.so
# With XSKNF_TIMELINE among the flags the variant carries the per-wave timeline.
set -e -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
OUT=$R/build/$NAME
mkdir -p "$OUT"
FLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-inline-asm -fvisibility=hidden --offload-arch=gfx950 -I$R/include"
cd "$R"
/opt/rocm/bin/hipcc $FLAGS "$@" --cuda-device-only -S -o "$OUT/checksummer-gfx950.s" xsknf_amd/csrc/checksummer.hip
python3 tools/check_inflight.py "$OUT/checksummer-gfx950.s"
/opt/rocm/bin/hipcc $FLAGS "$@" -shared -o "$OUT/libxsknf_gpu.so" xsknf_amd/csrc/checksummer.hip xsknf_amd/csrc/host_path.hip 2>&1 \
  | grep -v "argument unused" || true
test -f "$OUT/libxsknf_gpu.so"
