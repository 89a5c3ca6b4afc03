set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "tests $(date +%T)"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/d11_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/d11_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab.sh "lib" 2 "head em8 c2 c3" || exit 1
for kv in "RT_REFILL=40" "RT_REFILL=56" "RT_LEAF_MIN=16" "RT_LEAF_MIN=32"; do echo "== $kv"; env $kv bash tools/ab.sh "lib" 1 "head em8" || exit 1; done
