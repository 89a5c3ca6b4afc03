set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
RT_DIAG=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/e5_full.json 2> gpurun_out/e5_full.err
grep "rt diag\] step" gpurun_out/e5_full.err | tail -12
RT_DIAG=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --emulate 8 --emulate-rank 3 > gpurun_out/e5_e8.json 2> gpurun_out/e5_e8.err
grep "rt diag\] step" gpurun_out/e5_e8.err | tail -6
python3 -c "import json;d=json.load(open('gpurun_out/e5_e8.json'));print('e8', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['trace_share_of_step'])"
