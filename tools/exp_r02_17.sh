# shadow_step_kernel (soft-shadow samples advanced by a light kernel): parity tests, C4 A/B
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
echo "tests $(date +%T)"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/e17_gpu_tests.log 2>&1 || { tail -30 gpurun_out/e17_gpu_tests.log; exit 1; }
tail -1 gpurun_out/e17_gpu_tests.log
B="tests/golden/scenes/blend"
for F in 1 0 1 0; do
  RT_SHADOW_STEP=$F timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 --scene $B/glossy_reflection.json --light-radius 1.0 --light-samples 4 > gpurun_out/e17_c4_$F.json 2> gpurun_out/e17_c4_$F.err
  python3 -c "import json;d=json.load(open('gpurun_out/e17_c4_$F.json'));print('C4 shadow step $F', d['value'], d['ms_per_step'], d['roofline']['trace_share_of_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/e17_kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --scene $B/glossy_reflection.json --light-radius 1.0 --light-samples 4 > gpurun_out/e17_kt.json 2> gpurun_out/e17_kt.err
echo "done $(date +%T)"
