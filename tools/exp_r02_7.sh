set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
echo "tests $(date +%T)"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/e7_gpu_tests.log 2>&1 || { tail -30 gpurun_out/e7_gpu_tests.log; exit 1; }
tail -1 gpurun_out/e7_gpu_tests.log
timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/e7.json 2> gpurun_out/e7.err
python3 -c "import json;d=json.load(open('gpurun_out/e7.json'));print('tri1', d['value'], d['roofline']['avg_launch_ms'])"
RT_LIB_DIR=ray_tracying_amd/lib_pt timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 1 > gpurun_out/e7_pt.json 2> gpurun_out/e7_pt.err
grep "rt phase" gpurun_out/e7_pt.err | tail -1
