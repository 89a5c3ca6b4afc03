# fused shadows (auto on small calls): full GPU suite incl. test_gpu_fused
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/e44_gpu_tests.log 2>&1 || { tail -40 gpurun_out/e44_gpu_tests.log; exit 1; }
tail -1 gpurun_out/e44_gpu_tests.log
grep -E "fused|knobs" gpurun_out/e44_gpu_tests.log
echo "done $(date +%T)"
