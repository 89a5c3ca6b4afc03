set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/d8_head -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/d8_head.json 2> gpurun_out/d8_head.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/d8_em8 -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --emulate 8 --emulate-rank 7 > gpurun_out/d8_em8.json 2> gpurun_out/d8_em8.err || exit 1
