# BVH4 node layout A/B (AoS 64-B node per lane fetch vs SoA four 16-B arrays) and the plane
# test's t cut-off before the inside tests (lib, lib_soa: with it; lib_base: without)
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/e24_gpu_tests.log 2>&1 || { tail -30 gpurun_out/e24_gpu_tests.log; exit 1; }
tail -1 gpurun_out/e24_gpu_tests.log
RT_LIB_DIR=ray_tracying_amd/lib_soa timeout -k 10 600 python3 -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/e24_soa_tests.log 2>&1 || { tail -20 gpurun_out/e24_soa_tests.log; exit 1; }
tail -1 gpurun_out/e24_soa_tests.log
for V in lib lib_soa lib_base lib lib_soa lib_base; do
  RT_LIB_DIR=ray_tracying_amd/$V timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/e24_h_$V.json 2> gpurun_out/e24_h_$V.err
  python3 -c "import json;d=json.load(open('gpurun_out/e24_h_$V.json'));print('headline $V', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
echo "done $(date +%T)"
