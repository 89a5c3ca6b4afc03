# kernel timeline of the 8-way share with two slot pipelines (do the two streams overlap?)
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
RT_PIPES=2 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/e33_kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --emulate 8 --emulate-rank 7 > gpurun_out/e33_kt.json 2> gpurun_out/e33_kt.err
python3 tools/timeline.py gpurun_out/e33_kt 60 > gpurun_out/e33_timeline.txt
echo "done $(date +%T)"
