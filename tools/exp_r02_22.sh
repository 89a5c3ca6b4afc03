# kernel timelines: one rank's eighth of the headline frame, and C2 (primary rays only)
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/e22_e8 -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --emulate 8 --emulate-rank 7 > gpurun_out/e22_e8.json 2> gpurun_out/e22_e8.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/e22_c2 -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --primary-only --spp-sqrt 1 > gpurun_out/e22_c2.json 2> gpurun_out/e22_c2.err
RT_DIAG=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --emulate 8 --emulate-rank 7 > gpurun_out/e22_e8_diag.json 2> gpurun_out/e22_e8_diag.err
echo "done $(date +%T)"
