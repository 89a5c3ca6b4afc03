# nearest-first ordering as the default: full GPU suite, headline and 8-way share
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e48_gpu_tests.log 2>&1 || { tail -40 gpurun_out/e48_gpu_tests.log; exit 1; }
tail -1 gpurun_out/e48_gpu_tests.log
for E in "" "--emulate 8 --emulate-rank 7"; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 $E > gpurun_out/e48.json 2> gpurun_out/e48.err
  python3 -c "import json;d=json.load(open('gpurun_out/e48.json'));print('[$E]', d['value'], d['ms_per_step'])"
done
echo "done $(date +%T)"
