# camera rays alone (the soup without lights): full frame vs the 8-way share, with timelines
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for E in "" "--emulate 8 --emulate-rank 7"; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 --primary-only --spp-sqrt 10 $E > gpurun_out/e34.json 2> gpurun_out/e34.err || { tail -5 gpurun_out/e34.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/e34.json'));print('primary-only [$E]', d['value'], d['ms_per_step'], d['roofline']['trace_share_of_step'], d['config']['rays_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/e34_kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --primary-only --spp-sqrt 10 --emulate 8 --emulate-rank 7 > /dev/null 2> gpurun_out/e34_kt.err
python3 tools/timeline.py gpurun_out/e34_kt 12 > gpurun_out/e34_timeline.txt
echo "done $(date +%T)"
