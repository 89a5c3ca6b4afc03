set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
echo "smoke $(date +%T)"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1
echo "gpu tests $(date +%T)"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r03_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r03_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r03_gpu_tests.log
bash tools/ab.sh "lib" 1 "head c2"
