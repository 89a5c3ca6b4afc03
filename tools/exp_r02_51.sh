# slots in flight for the whole headline frame, current build: 16M (default) / 24M / 32M
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for rep in 1 2; do
  for S in 16777216 25165824 33554432; do
    RT_SLOTS=$S timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/e51.json 2> gpurun_out/e51.err
    python3 -c "import json;d=json.load(open('gpurun_out/e51.json'));print('slots $S', d['value'], d['ms_per_step'], d['roofline']['launches_per_step'], d['roofline']['trace_share_of_step'])"
  done
done
echo "done $(date +%T)"
