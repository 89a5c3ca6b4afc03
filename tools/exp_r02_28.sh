# start_kernel as a grid of flag-scanning waves: parity tests, then headline / C3 / C4 A/B vs lib_base (both one pipeline)
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
echo "tests $(date +%T)"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/e28_gpu_tests.log 2>&1 || { tail -30 gpurun_out/e28_gpu_tests.log; exit 1; }
tail -1 gpurun_out/e28_gpu_tests.log
export RT_PIPES=1
B="tests/golden/scenes/blend"
for V in lib lib_base lib lib_base; do
  RT_LIB_DIR=ray_tracying_amd/$V timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/e28_h_$V.json 2> gpurun_out/e28_h_$V.err
  python3 -c "import json;d=json.load(open('gpurun_out/e28_h_$V.json'));print('headline $V', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
for V in lib lib_base; do
  RT_LIB_DIR=ray_tracying_amd/$V timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 3 --scene $B/Antialiasing.json > gpurun_out/e28_c3_$V.json 2> gpurun_out/e28_c3_$V.err
  python3 -c "import json;d=json.load(open('gpurun_out/e28_c3_$V.json'));print('C3 $V', d['value'], d['ms_per_step'], d['roofline']['trace_share_of_step'])"
  RT_LIB_DIR=ray_tracying_amd/$V timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 --scene $B/glossy_reflection.json --light-radius 1.0 --light-samples 4 > gpurun_out/e28_c4_$V.json 2> gpurun_out/e28_c4_$V.err
  python3 -c "import json;d=json.load(open('gpurun_out/e28_c4_$V.json'));print('C4 $V', d['value'], d['ms_per_step'], d['roofline']['trace_share_of_step'])"
done
echo "done $(date +%T)"
for V in lib lib_base; do
  RT_LIB_DIR=ray_tracying_amd/$V timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 10 --primary-only --spp-sqrt 1 > gpurun_out/e28_c2_$V.json 2> gpurun_out/e28_c2_$V.err
  python3 -c "import json;d=json.load(open('gpurun_out/e28_c2_$V.json'));print('C2 $V', d['value'], d['ms_per_step'])"
  RT_LIB_DIR=ray_tracying_amd/$V timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 10 --emulate 8 --emulate-rank 7 > gpurun_out/e28_e8_$V.json 2> gpurun_out/e28_e8_$V.err
  python3 -c "import json;d=json.load(open('gpurun_out/e28_e8_$V.json'));print('8-way share $V', d['value'], d['ms_per_step'])"
done
