# fused shadows A/B, same box, alternating: 8-way and 4-way shares
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for rep in 1 2 3; do
  for F in 0 1; do
    for E in "--emulate 8 --emulate-rank 7" "--emulate 4 --emulate-rank 3"; do
      RT_FUSE=$F timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 $E > gpurun_out/e43.json 2> gpurun_out/e43.err || { tail -5 gpurun_out/e43.err; exit 1; }
      python3 -c "import json;d=json.load(open('gpurun_out/e43.json'));print('fuse $F [$E]', d['value'], d['ms_per_step'])"
    done
  done
done
echo "done $(date +%T)"
