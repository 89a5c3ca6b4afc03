set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for m in 1 2 3; do
  echo "merge $m $(date +%T)"
  RT_LEAF_MERGE=$m timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/e3_m$m.json 2> gpurun_out/e3_m$m.err
  python3 -c "import json;d=json.load(open('gpurun_out/e3_m$m.json'));print('m$m', d['value'], d['roofline']['avg_launch_ms'])"; grep instrumented gpurun_out/e3_m$m.err
done
