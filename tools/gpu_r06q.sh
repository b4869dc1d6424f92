set -o pipefail
OUT=gpurun_out/${1:-r06q}; mkdir -p $OUT
timeout -k 10 400 python -u tools/nf_start_probe.py --starts 200 --hold 0.3 --out $OUT/nf_start_probe.jsonl > $OUT/nf_start_probe.log 2>&1 || { echo probe failed; tail -20 $OUT/nf_start_probe.log; exit 1; }
tail -1 $OUT/nf_start_probe.log
