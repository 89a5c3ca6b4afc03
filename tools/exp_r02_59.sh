# fused-path parity additions (textured planes, soft samples on planes) + full GPU suite
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/e59_gpu_tests.log 2>&1 || { tail -40 gpurun_out/e59_gpu_tests.log; exit 1; }
tail -1 gpurun_out/e59_gpu_tests.log
echo "done $(date +%T)"
