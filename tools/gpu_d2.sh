set -o pipefail
mkdir -p gpurun_out
for dh in 1 0; do
RT_DRAIN_HELP=$dh RT_LIB_DIR=ray_tracying_amd/lib_et timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --primary-only --spp-sqrt 1 > gpurun_out/d2_c2_$dh.json 2> gpurun_out/d2_c2_$dh.err || exit 1
grep "rt exit" gpurun_out/d2_c2_$dh.err | tail -2
RT_DRAIN_HELP=$dh RT_LIB_DIR=ray_tracying_amd/lib_et timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --emulate 8 --emulate-rank 7 > gpurun_out/d2_em8_$dh.json 2> gpurun_out/d2_em8_$dh.err || exit 1
grep "rt exit" gpurun_out/d2_em8_$dh.err | tail -3
done
