# fused point-light shadows on whole soup frames, current build: headline and C5 (1 GPU), RT_FUSE=0/1
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for F in 0 1; do
  RT_FUSE=$F timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/e56.json 2> gpurun_out/e56.err
  python3 -c "import json;d=json.load(open('gpurun_out/e56.json'));print('fuse $F headline', d['value'], d['ms_per_step'], d['roofline']['launches_per_step'])"
done
for F in 0 1; do
  RT_FUSE=$F timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --res 4096 --spp-sqrt 8 > gpurun_out/e56.json 2> gpurun_out/e56.err
  python3 -c "import json;d=json.load(open('gpurun_out/e56.json'));print('fuse $F C5', d['value'], d['ms_per_step'], d['roofline']['launches_per_step'])"
done
echo "done $(date +%T)"
