# reflection-only instance of the frames logic kernel (4 waves/SIMD): GPU suite, then C4 / C3 A/B
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
B=tests/golden/scenes/blend
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e52_gpu_tests.log 2>&1 || { tail -40 gpurun_out/e52_gpu_tests.log; exit 1; }
tail -1 gpurun_out/e52_gpu_tests.log
for rep in 1 2; do
  for V in lib_prev lib; do
    RT_LIB_DIR=ray_tracying_amd/$V timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 --scene $B/glossy_reflection.json --light-radius 1.0 --light-samples 4 > gpurun_out/e52_c4.json 2> gpurun_out/e52_c4.err
    python3 -c "import json;d=json.load(open('gpurun_out/e52_c4.json'));print('$V C4', d['value'], d['ms_per_step'], d['roofline']['trace_share_of_step'])"
  done
done
echo "done $(date +%T)"
