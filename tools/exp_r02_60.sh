# pinhole camera queries without a stored origin: GPU suite, then A/B (previous commit vs this)
# on the headline, the 8-way share, C3 and C4
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
B=tests/golden/scenes/blend
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/e60_gpu_tests.log 2>&1 || { tail -40 gpurun_out/e60_gpu_tests.log; exit 1; }
tail -1 gpurun_out/e60_gpu_tests.log
for rep in 1 2; do
  for V in lib_prev lib; do
    for E in "" "--emulate 8 --emulate-rank 7"; do
      RT_LIB_DIR=ray_tracying_amd/$V timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 $E > gpurun_out/e60.json 2> gpurun_out/e60.err
      python3 -c "import json;d=json.load(open('gpurun_out/e60.json'));print('$V [$E]', d['value'], d['ms_per_step'])"
    done
    RT_LIB_DIR=ray_tracying_amd/$V timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --scene $B/Antialiasing.json > gpurun_out/e60_c3.json 2> gpurun_out/e60_c3.err
    python3 -c "import json;d=json.load(open('gpurun_out/e60_c3.json'));print('$V C3', d['value'], d['ms_per_step'])"
    RT_LIB_DIR=ray_tracying_amd/$V timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 --scene $B/glossy_reflection.json --light-radius 1.0 --light-samples 4 > gpurun_out/e60_c4.json 2> gpurun_out/e60_c4.err
    python3 -c "import json;d=json.load(open('gpurun_out/e60_c4.json'));print('$V C4', d['value'], d['ms_per_step'])"
  done
done
echo "done $(date +%T)"
