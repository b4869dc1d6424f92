set -o pipefail
OUT=gpurun_out/r06c; mkdir -p $OUT
for args in "1048576 " "8388608 " "1048576 68719476736" "8388608 68719476736" "8388608 4294967296" "8388608 2147483648"; do
  set -- $args
  if [ -n "$2" ]; then export XSKNF_MULTI_P2P_PIECE=$2; else unset XSKNF_MULTI_P2P_PIECE; fi
  timeout -k 10 200 python -u tools/diag_multi_p2p.py $1 2>&1 | grep -v amdgpu.ids | grep '^{' | tee -a $OUT/diag.jsonl || exit 1
done
