# refill / leaf thresholds: default vs leaf 20 + refill 40, alternating, 3 reps (headline)
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for rep in 1 2 3; do
  for cfg in "RT_LEAF_MIN=16 RT_REFILL=48" "RT_LEAF_MIN=20 RT_REFILL=40" "RT_LEAF_MIN=20 RT_REFILL=48"; do
    env $cfg timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/e58.json 2> gpurun_out/e58.err
    python3 -c "import json;d=json.load(open('gpurun_out/e58.json'));print('$cfg', d['value'], d['ms_per_step'])"
  done
done
echo "done $(date +%T)"
