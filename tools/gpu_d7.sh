set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "tests $(date +%T)"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/d7_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/d7_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab.sh "lib" 1 "head c2 em8 em4 c3" || exit 1
echo "== RT_FUSE=0"; RT_FUSE=0 bash tools/ab.sh "lib" 1 "head" || exit 1
echo "== RT_TILE_ORDER=0"; RT_TILE_ORDER=0 bash tools/ab.sh "lib" 1 "head" || exit 1
