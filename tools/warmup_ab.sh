mkdir -p gpurun_out/warm
for w in 0.1 3 0.1 3; do
  timeout -k 10 120 python bench.py --secondary "" --cpu-seconds 0 --no-verify --min-warmup-s $w > gpurun_out/warm/w$w.$RANDOM.json 2>/dev/null || exit 1
done
