set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for kv in "RT_PIPES=2" "RT_PIPES=1"; do
  echo "== $kv"
  env $kv bash tools/ab.sh "lib" 1 "em2 em4 em8 head c3 c4 c5" || exit 1
done
for kv in "RT_TRACE_BPC=4" "RT_TRACE_BPC=5" "RT_TRACE_BPC=6"; do
  echo "== $kv"
  env $kv bash tools/ab.sh "lib" 1 "c2 em8" || exit 1
done
