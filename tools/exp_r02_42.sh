# fused point-light shadow rays (trace_refill_kernel<.., kFuse>): GPU tests, then RT_FUSE=0/1 on
# the headline and the 8/4/2-way shares
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e42_gpu_tests.log 2>&1 || { tail -30 gpurun_out/e42_gpu_tests.log; exit 1; }
tail -1 gpurun_out/e42_gpu_tests.log
for F in 0 1; do
  for E in "" "--emulate 8 --emulate-rank 7" "--emulate 4 --emulate-rank 3" "--emulate 2 --emulate-rank 1"; do
    RT_FUSE=$F timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 $E > gpurun_out/e42.json 2> gpurun_out/e42.err || { tail -5 gpurun_out/e42.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/e42.json'));print('fuse $F [$E]', d['value'], d['ms_per_step'], d['roofline']['launches_per_step'], d['roofline']['trace_share_of_step'])"
  done
done
echo "done $(date +%T)"
