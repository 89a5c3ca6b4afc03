# host overhead per rt_render_tiles call (event wait: blocking vs spin), 8-way share
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python3 tools/host_gap.py 8 30
RT_SPIN_WAIT=1 timeout -k 10 300 python3 tools/host_gap.py 8 30
for S in 0 1; do
  RT_SPIN_WAIT=$S timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --emulate 8 --emulate-rank 7 > gpurun_out/e37.json 2> gpurun_out/e37.err || { tail -5 gpurun_out/e37.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/e37.json'));print('spin $S share8', d['value'], d['ms_per_step'])"
done
echo "done $(date +%T)"
