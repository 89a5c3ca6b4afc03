# reduce_kernel staging chunk (samples per pixel per LDS pass): 16 (default) / 8 / 4, with kernel stats
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
RT_LIB_DIR=ray_tracying_amd/lib_rc8 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py -x -q --timeout 120 --timeout-method thread > gpurun_out/e29_rc8_tests.log 2>&1 || { tail -20 gpurun_out/e29_rc8_tests.log; exit 1; }
tail -1 gpurun_out/e29_rc8_tests.log
for V in lib lib_rc8 lib_rc4; do
  RT_LIB_DIR=ray_tracying_amd/$V timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/e29_$V -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/e29_$V.json 2> gpurun_out/e29_$V.err
  python3 -c "import json;d=json.load(open('gpurun_out/e29_$V.json'));print('headline $V', d['value'], d['ms_per_step'])"
  grep -h reduce_kernel gpurun_out/e29_$V/*kernel_stats.csv | cut -d, -f1-4
done
echo "done $(date +%T)"
