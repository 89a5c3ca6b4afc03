# host-loop trim (init does the resets, first step without logic, trace writes the host flag,
# reduce + stats copy per host batch, tile list cached, 128 claim shards): tests, benches, timeline
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e36_gpu_tests.log 2>&1 || { tail -30 gpurun_out/e36_gpu_tests.log; exit 1; }
tail -1 gpurun_out/e36_gpu_tests.log
for E in "" "--emulate 8 --emulate-rank 7" "--emulate 4 --emulate-rank 3" "--emulate 2 --emulate-rank 1"; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 $E > gpurun_out/e36.json 2> gpurun_out/e36.err || { tail -5 gpurun_out/e36.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/e36.json'));print('[$E]', d['value'], d['ms_per_step'], d['roofline']['trace_share_of_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/e36_kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --emulate 8 --emulate-rank 7 > /dev/null 2> gpurun_out/e36_kt.err
echo "done $(date +%T)"
