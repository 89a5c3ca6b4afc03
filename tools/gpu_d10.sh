set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in "em8:--emulate 8 --emulate-rank 7" "head:" "c2:--primary-only --spp-sqrt 1"; do
  n=${w%%:*}; a=${w#*:}
  RT_LIB_DIR=ray_tracying_amd/lib_et timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 $a > gpurun_out/d10_$n.json 2> gpurun_out/d10_$n.err || exit 1
  echo $n; grep "rt exit" gpurun_out/d10_$n.err | tail -2
done
