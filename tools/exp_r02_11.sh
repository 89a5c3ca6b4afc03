# query record AoS: parity tests, bench; logic kernel at 4 waves/SIMD (variant lw4) A/B
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
echo "tests $(date +%T)"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/e11_gpu_tests.log 2>&1 || { tail -30 gpurun_out/e11_gpu_tests.log; exit 1; }
tail -1 gpurun_out/e11_gpu_tests.log
for V in lib lib_lw4 lib lib_lw4; do
  RT_LIB_DIR=ray_tracying_amd/$V timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/e11_$V.json 2> gpurun_out/e11_$V.err
  python3 -c "import json;d=json.load(open('gpurun_out/e11_$V.json'));print('$V', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
echo "done $(date +%T)"
