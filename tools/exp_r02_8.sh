# two slot pipelines on two streams: parity tests, then bench A/B (RT_PIPES=1 vs 2) + kernel trace
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
echo "tests $(date +%T)"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/e8_gpu_tests.log 2>&1 || { tail -30 gpurun_out/e8_gpu_tests.log; exit 1; }
tail -1 gpurun_out/e8_gpu_tests.log
for P in 1 2; do
  RT_PIPES=$P timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/e8_p$P.json 2> gpurun_out/e8_p$P.err
  python3 -c "import json;d=json.load(open('gpurun_out/e8_p$P.json'));print('pipes $P', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/e8_kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/e8_kt.json 2> gpurun_out/e8_kt.err
echo "done $(date +%T)"
