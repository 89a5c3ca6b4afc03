set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for kv in "X=1" "RT_PIPES=1" "RT_FUSE=0" "RT_LEAF_MIN=16" "RT_LEAF_MIN=32" "RT_TRACE_BPC=5"; do
  echo "== $kv"
  env $kv bash tools/ab.sh "lib" 1 "em8 c2" || exit 1
done
