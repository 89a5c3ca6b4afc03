# fused point-light shadow rays for transformed shapes and small scenes: GPU suite, then C3 with
# RT_FUSE=0 vs default, C4 and the headline once
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
B=tests/golden/scenes/blend
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/e54_gpu_tests.log 2>&1 || { tail -40 gpurun_out/e54_gpu_tests.log; exit 1; }
tail -1 gpurun_out/e54_gpu_tests.log
for rep in 1 2; do
  for F in 0 1; do
    RT_FUSE=$F timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --scene $B/Antialiasing.json > gpurun_out/e54_c3.json 2> gpurun_out/e54_c3.err
    python3 -c "import json;d=json.load(open('gpurun_out/e54_c3.json'));print('fuse $F C3', d['value'], d['ms_per_step'], d['roofline']['trace_share_of_step'], d['roofline']['launches_per_step'])"
  done
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 --scene $B/glossy_reflection.json --light-radius 1.0 --light-samples 4 > gpurun_out/e54_c4.json 2> gpurun_out/e54_c4.err
python3 -c "import json;d=json.load(open('gpurun_out/e54_c4.json'));print('C4', d['value'], d['ms_per_step'])"
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/e54.json 2> gpurun_out/e54.err
python3 -c "import json;d=json.load(open('gpurun_out/e54.json'));print('headline', d['value'], d['ms_per_step'])"
echo "done $(date +%T)"
