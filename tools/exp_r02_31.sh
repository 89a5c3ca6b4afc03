# kernel timeline of one headline frame (compare with the 8-way share's, exp_r02_30)
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/e31_kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/e31_kt.json 2> gpurun_out/e31_kt.err
python3 tools/timeline.py gpurun_out/e31_kt 80 > gpurun_out/e31_timeline.txt
echo "done $(date +%T)"
