set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
echo "gpu tests $(date +%T)"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r03_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r03_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r03_gpu_tests.log
RT_LIB_DIR=ray_tracying_amd/lib_pt timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/r03_pt.json 2> gpurun_out/r03_pt.err
grep "rt phase" gpurun_out/r03_pt.err | tail -3
RT_DIAG=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/r03_diag.json 2> gpurun_out/r03_diag.err
grep "rt diag" gpurun_out/r03_diag.err | tail -14
bash tools/ab.sh lib 1 "head em8 c2"
