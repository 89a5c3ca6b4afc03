set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/d3_em8 -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 --emulate 8 --emulate-rank 7 > gpurun_out/d3_em8.json 2> gpurun_out/d3_em8.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/d3_c2 -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 --primary-only --spp-sqrt 1 > gpurun_out/d3_c2.json 2> gpurun_out/d3_c2.err || exit 1
find gpurun_out/d3_em8 gpurun_out/d3_c2 -name "*.csv" | head
