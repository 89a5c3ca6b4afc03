# C2, one rank's share of 2/4/8-way splits, and C5 (one GPU, rank 3 of 8) on the current build.
set -eo pipefail
L=${1:?label}
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --primary-only --spp-sqrt 1 > gpurun_out/${L}_c2_primary_only_bench.json 2> gpurun_out/${L}_c2.err
for N in 2 4 8; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --emulate $N --emulate-rank $((N - 1)) > gpurun_out/${L}_emulated_share_of_${N}_bench.json 2> gpurun_out/${L}_em$N.err
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --res 4096 --spp-sqrt 8 > gpurun_out/${L}_c5_4096_64spp_1gpu_bench.json 2> gpurun_out/${L}_c5.err
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --res 4096 --spp-sqrt 8 --emulate 8 --emulate-rank 3 > gpurun_out/${L}_c5_emulated_rank3_of_8_bench.json 2> gpurun_out/${L}_c5e.err
echo "done $(date +%T)"
