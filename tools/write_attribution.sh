#!/bin/bash
# Attribution of the headline trace launch's HBM writes (run on the GPU box through gpurun):
#   make variant V=wd VDEFS=-DRT_WRITE_DIAG   (here, before the call)
#   bash tools/write_attribution.sh LABEL
# The RT_WRITE_DIAG build's store counts per kind (HBM stack entries, result words, hit
# records, occlusion words), and PMC WRITE_SIZE of the default build at 7 and 6 waves/SIMD
# and with the LDS stack cut to 8 entries (more entries spill to the HBM stack area).
source tools/gpu_steps.sh
L=${1:?label}
RT_LIB_DIR=ray_tracying_amd/lib_wd step ${L}_wd7.log 200 python3 bench.py --no-cpu-baseline --steps 1 --warmup 0
RT_LIB_DIR=ray_tracying_amd/lib_wd RT_TRACE_SEVEN=0 step ${L}_wd6.log 200 python3 bench.py --no-cpu-baseline --steps 1 --warmup 0
RT_LIB_DIR=ray_tracying_amd/lib_wd RT_LDS_STACK=8 step ${L}_wd7_s8.log 200 python3 bench.py --no-cpu-baseline --steps 1 --warmup 0
for v in "w7" "w6:RT_TRACE_SEVEN=0" "w7s8:RT_LDS_STACK=8" "w6s8:RT_TRACE_SEVEN=0 RT_LDS_STACK=8"; do
  tag=${v%%:*}; envs=""; [ "$tag" != "$v" ] && envs=${v#*:}
  step ${L}_pmcW_${tag}.log 120 env $envs rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${L}_pmcW_${tag} -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0
done
