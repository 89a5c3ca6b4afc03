# fused point-light shadow rays in the trace kernel: parity tests, bench A/B, kernel trace
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
echo "tests $(date +%T)"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/e10_gpu_tests.log 2>&1 || { tail -30 gpurun_out/e10_gpu_tests.log; exit 1; }
tail -1 gpurun_out/e10_gpu_tests.log
for F in 1 0 1; do
  RT_FUSE_SHADOWS=$F timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/e10_f$F.json 2> gpurun_out/e10_f$F.err
  python3 -c "import json;d=json.load(open('gpurun_out/e10_f$F.json'));print('fuse $F', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['launches_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/e10_kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/e10_kt.json 2> gpurun_out/e10_kt.err
echo "done $(date +%T)"
