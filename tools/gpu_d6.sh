set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for kv in "RT_SLOTS=33554432" "X=1" "RT_SLOTS=67108864" "RT_SLOTS=110000000"; do echo "== head $kv"; env $kv bash tools/ab.sh "lib" 1 "head" || exit 1; done
for kv in "X=1" "RT_SLOTS=54525952"; do echo "== em2 $kv"; env $kv bash tools/ab.sh "lib" 1 "em2" || exit 1; done
for kv in "X=1" "RT_SLOTS=134217728" "RT_SLOTS=201326592"; do echo "== c5 $kv"; env $kv bash tools/ab.sh "lib" 1 "c5" || exit 1; done
for kv in "X=1" "RT_SLOTS=33554432" "RT_SLOTS=8388608"; do echo "== c4 $kv"; env $kv bash tools/ab.sh "lib" 1 "c4" || exit 1; done
for kv in "X=1" "RT_SLOTS=33554432" "RT_SLOTS=67108864"; do echo "== c3 $kv"; env $kv bash tools/ab.sh "lib" 1 "c3" || exit 1; done
