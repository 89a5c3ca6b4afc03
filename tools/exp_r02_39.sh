# trace launch drain (RT_EXIT_TIMING build): when the work queue runs dry vs when the waves exit
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
RT_LIB_DIR=ray_tracying_amd/lib_exit timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > /dev/null 2> gpurun_out/e39_full.err
RT_LIB_DIR=ray_tracying_amd/lib_exit timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --emulate 8 --emulate-rank 7 > /dev/null 2> gpurun_out/e39_share.err
grep "rt exit" gpurun_out/e39_full.err | tail -10
echo ---
grep "rt exit" gpurun_out/e39_share.err | tail -2
echo "done $(date +%T)"
