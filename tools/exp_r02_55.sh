# a closest hit starts its soft shade loop in the tracing lane: GPU suite, then C4 with
# RT_SOFT_START=0 vs default, and the headline (unaffected) once
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
B=tests/golden/scenes/blend
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/e55_gpu_tests.log 2>&1 || { tail -40 gpurun_out/e55_gpu_tests.log; exit 1; }
tail -1 gpurun_out/e55_gpu_tests.log
for rep in 1 2; do
  for F in 0 1; do
    RT_SOFT_START=$F timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 --scene $B/glossy_reflection.json --light-radius 1.0 --light-samples 4 > gpurun_out/e55_c4.json 2> gpurun_out/e55_c4.err
    python3 -c "import json;d=json.load(open('gpurun_out/e55_c4.json'));print('start $F C4', d['value'], d['ms_per_step'], d['roofline']['trace_share_of_step'], d['roofline']['launches_per_step'])"
  done
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/e55.json 2> gpurun_out/e55.err
python3 -c "import json;d=json.load(open('gpurun_out/e55.json'));print('headline', d['value'], d['ms_per_step'])"
echo "done $(date +%T)"
