# straggler retry (RT_RETRY_US): parity under aggressive settings, then headline / 8-way share sweeps
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for R in 1 20; do
  RT_RETRY_US=$R timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_knobs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/e40_tests_$R.log 2>&1 || { tail -30 gpurun_out/e40_tests_$R.log; exit 1; }
  echo "retry $R: $(tail -1 gpurun_out/e40_tests_$R.log)"
done
for R in 0 30 60 100 200; do
  for E in "" "--emulate 8 --emulate-rank 7"; do
    RT_RETRY_US=$R timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 $E > gpurun_out/e40.json 2> gpurun_out/e40.err || { tail -5 gpurun_out/e40.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/e40.json'));print('retry $R [$E]', d['value'], d['ms_per_step'], d['roofline']['launches_per_step'])"
  done
done
echo "done $(date +%T)"
