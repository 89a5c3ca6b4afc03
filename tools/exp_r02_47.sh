# node-visit sort network: 5 compare-exchanges (full sort) vs 4 (middle pair unordered) vs 3
# (nearest only): parity of the partial sorts, then the headline, alternating, with node visits
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for V in lib_sort4 lib_sort3; do
  RT_LIB_DIR=ray_tracying_amd/$V timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py -x -q --timeout 120 --timeout-method thread > gpurun_out/e47_$V.log 2>&1 || { tail -20 gpurun_out/e47_$V.log; exit 1; }
  echo "$V: $(tail -1 gpurun_out/e47_$V.log)"
done
for rep in 1 2; do
  for V in lib lib_sort4 lib_sort3; do
    RT_LIB_DIR=ray_tracying_amd/$V timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/e47.json 2> gpurun_out/e47.err || { tail -5 gpurun_out/e47.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/e47.json'));print('$V', d['value'], d['ms_per_step'])"
    grep -o "node visits [0-9]* ([0-9.]*/ray)" gpurun_out/e47.err
  done
done
echo "done $(date +%T)"
