set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for kv in "X=1" "RT_TRACE_BPC=5" "RT_TRACE_BPC=4"; do echo "== $kv"; env $kv bash tools/ab.sh "lib" 1 "em8 em4" || exit 1; done
done
