# r05: attribution of the headline trace launch's HBM writes -- the store
# counts of an RT_WRITE_DIAG build (lib_wd), and PMC WRITE_SIZE of the default build at 7 and 6
# waves/SIMD and with a shallower LDS stack (more entries spill to the HBM stack area)
source tools/gpu_steps.sh
RT_LIB_DIR=ray_tracying_amd/lib_wd step r05p_wd7.log 200 python3 bench.py --no-cpu-baseline --steps 1 --warmup 0
RT_LIB_DIR=ray_tracying_amd/lib_wd RT_TRACE_SEVEN=0 step r05p_wd6.log 200 python3 bench.py --no-cpu-baseline --steps 1 --warmup 0
RT_LIB_DIR=ray_tracying_amd/lib_wd RT_LDS_STACK=8 step r05p_wd7_s8.log 200 python3 bench.py --no-cpu-baseline --steps 1 --warmup 0
for v in "w7" "w6:RT_TRACE_SEVEN=0" "w7s8:RT_LDS_STACK=8" "w6s8:RT_TRACE_SEVEN=0 RT_LDS_STACK=8"; do
  tag=${v%%:*}; envs=""; [ "$tag" != "$v" ] && envs=${v#*:}
  step r05p_pmcW_${tag}.log 120 env $envs rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r05p_pmcW_${tag} -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0
  python3 tools/pmc_traffic.py --write gpurun_out/r05p_pmcW_${tag} --fetch gpurun_out/r05p_pmcW_${tag} --kernel "trace_refill_kernel<false" --out gpurun_out/r05p_pmcW_${tag}.json --label "$tag" > /dev/null || true
  grep write_bytes gpurun_out/r05p_pmcW_${tag}.json || true
done
