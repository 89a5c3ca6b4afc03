# SLP vectoriser off for the device code (-fno-slp-vectorize: the headline trace kernel drops
# from 125 to 84 VGPRs -- no register pairs built for v_pk_add/v_pk_mul -- so 5 waves/SIMD fit
# without spills): default vs noslp (waves target 4) vs noslp5 vs noslp6; alternating, 2 reps
# (headline), C4 default vs noslp, then the GPU parity suite on the noslp build.
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for rep in 1 2; do
  for lib in lib lib_noslp lib_noslp5 lib_noslp6; do
    RT_LIB_DIR=ray_tracying_amd/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/e61.json 2> gpurun_out/e61_$lib.err
    python3 -c "import json;d=json.load(open('gpurun_out/e61.json'));print('$lib', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done
for lib in lib lib_noslp lib_noslp5; do
  RT_LIB_DIR=ray_tracying_amd/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 --scene tests/golden/scenes/blend/glossy_reflection.json --light-radius 1.0 --light-samples 4 > gpurun_out/e61c4.json 2> gpurun_out/e61c4.err
  python3 -c "import json;d=json.load(open('gpurun_out/e61c4.json'));print('C4 $lib', d['value'], d['ms_per_step'])"
done
RT_LIB_DIR=ray_tracying_amd/lib_noslp5 timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/e61_gpu_tests.log 2>&1 || { tail -40 gpurun_out/e61_gpu_tests.log; exit 1; }
tail -1 gpurun_out/e61_gpu_tests.log
echo "done $(date +%T)"
