set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "tests $(date +%T)"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/d9_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/d9_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab.sh "lib lib_prev" 2 "head em8 c2" || exit 1
bash tools/measure_r03_shares.sh r03_v7 || exit 1
