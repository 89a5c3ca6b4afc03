# batch-claim shard count: headline and the 8-way share (start_kernel claim atomics)
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for S in 32 128 512 1024; do
  for E in "" "--emulate 8 --emulate-rank 7"; do
    RT_BATCH_SHARDS=$S timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 $E > gpurun_out/e35.json 2> gpurun_out/e35.err || { tail -5 gpurun_out/e35.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/e35.json'));print('shards $S [$E]', d['value'], d['ms_per_step'], d['roofline']['trace_share_of_step'])"
  done
done
RT_BATCH_SHARDS=1024 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/e35_kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --emulate 8 --emulate-rank 7 > /dev/null 2> gpurun_out/e35_kt.err
python3 tools/timeline.py gpurun_out/e35_kt 14 > gpurun_out/e35_timeline.txt
echo "done $(date +%T)"
