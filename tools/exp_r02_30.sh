# emulated 8-way share of the headline (rank 7/8): slot count and pipeline count, plus a kernel
# timeline of one frame
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
B="python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 --emulate 8 --emulate-rank 7"
for cfg in "RT_PIPES=1" "RT_PIPES=2" "RT_SLOTS=8388608" "RT_SLOTS=4194304" "RT_PIPES=2 RT_SLOTS=8388608" "RT_PIPES=1"; do
  env $cfg timeout -k 10 300 $B > gpurun_out/e30.json 2> gpurun_out/e30.err || { tail -5 gpurun_out/e30.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/e30.json'));print('share8 $cfg', d['value'], d['ms_per_step'], d['roofline']['trace_share_of_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/e30_kt -o kt --output-format csv -- $B --steps 1 > gpurun_out/e30_kt.json 2> gpurun_out/e30_kt.err
python3 tools/timeline.py gpurun_out/e30_kt 400 > gpurun_out/e30_timeline.txt
echo "done $(date +%T)"
