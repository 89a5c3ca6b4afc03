# refill / leaf thresholds re-swept on the current build (headline)
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for cfg in "RT_LEAF_MIN=16 RT_REFILL=48" "RT_LEAF_MIN=12" "RT_LEAF_MIN=20" "RT_LEAF_MIN=24" "RT_REFILL=40" "RT_REFILL=56" "RT_LEAF_MIN=16 RT_REFILL=48"; do
  env $cfg timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/e57.json 2> gpurun_out/e57.err
  python3 -c "import json;d=json.load(open('gpurun_out/e57.json'));print('$cfg', d['value'], d['ms_per_step'])"
done
echo "done $(date +%T)"
