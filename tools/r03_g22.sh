set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
echo "gpu tests $(date +%T)"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r03_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r03_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r03_gpu_tests.log
for r in 1 2; do bash tools/ab.sh "lib lib_base" 1 "c2 c3"; done
