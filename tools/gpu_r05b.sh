# r05 A/B of the hit record written once at settle (lib) against the commit before (lib_prev):
# GPU tests on lib, same-box bench pairs, WRITE_SIZE of both, the phase-timing build.
source tools/gpu_steps.sh
step r05b_gpu_tests.log 1200 python3 -u -m pytest tests -m gpu -x -q --timeout 800 --timeout-method thread
step r05b_ab.txt 900 bash tools/ab.sh "lib lib_prev" 2 "head em8 c5 c3"
for L in lib lib_prev; do
  step r05b_pmcW_$L.log 200 env RT_LIB_DIR=ray_tracying_amd/$L rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r05b_pmcW_$L -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0
  step r05b_pmcF_$L.log 200 env RT_LIB_DIR=ray_tracying_amd/$L rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r05b_pmcF_$L -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0
  python3 tools/pmc_traffic.py --fetch gpurun_out/r05b_pmcF_$L --write gpurun_out/r05b_pmcW_$L --kernel "trace_refill_kernel<false" --out gpurun_out/r05b_${L}_pmc_traffic.json --label "r05b $L" > /dev/null
done
step r05b_phase.log 200 env RT_LIB_DIR=ray_tracying_amd/lib_phase python3 bench.py --no-cpu-baseline --steps 2 --warmup 0
