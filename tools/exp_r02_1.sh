set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/pmc_passes.sh diag1 tools/pmc_sets_diag.txt
for bpc in 2 3; do echo "bpc $bpc $(date +%T)"; RT_TRACE_BPC=$bpc timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/e1_bpc$bpc.json 2> gpurun_out/e1_bpc$bpc.err; done
echo "w5 $(date +%T)"; RT_LIB_DIR=ray_tracying_amd/lib_w5 timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/e1_w5.json 2> gpurun_out/e1_w5.err
echo "lds8 $(date +%T)"; RT_LDS_STACK=8 timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/e1_lds8.json 2> gpurun_out/e1_lds8.err
echo "w5 lds12 $(date +%T)"; RT_LDS_STACK=12 RT_LIB_DIR=ray_tracying_amd/lib_w5 timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/e1_w5_lds12.json 2> gpurun_out/e1_w5_lds12.err
echo done
