# per-step queries and trace rate (RT_DIAG): headline frame vs the 8-way share
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
RT_DIAG=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > /dev/null 2> gpurun_out/e38_full.err
RT_DIAG=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --emulate 8 --emulate-rank 7 > /dev/null 2> gpurun_out/e38_share.err
grep "rt diag" gpurun_out/e38_full.err | tail -14
echo ---
grep "rt diag" gpurun_out/e38_share.err | tail -6
echo "done $(date +%T)"
