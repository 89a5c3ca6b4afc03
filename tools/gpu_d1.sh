set -o pipefail
mkdir -p gpurun_out
echo "tests $(date +%T)"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/d1_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/d1_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
echo "ab $(date +%T)"
bash tools/ab.sh "lib lib_base" 2 "em8 c2 head" && RT_DRAIN_HELP=0 bash tools/ab.sh "lib" 1 "em8 c2"
