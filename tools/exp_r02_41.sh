# same-box A/B: previous commit's kernels (lib_head) vs the host-loop trim (lib), headline and 8-way share
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for rep in 1 2; do
  for V in lib_head lib; do
    for E in "" "--emulate 8 --emulate-rank 7"; do
      RT_LIB_DIR=ray_tracying_amd/$V timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 $E > gpurun_out/e41.json 2> gpurun_out/e41.err || { tail -5 gpurun_out/e41.err; exit 1; }
      python3 -c "import json;d=json.load(open('gpurun_out/e41.json'));print('$V [$E]', d['value'], d['ms_per_step'])"
    done
  done
done
echo "done $(date +%T)"
