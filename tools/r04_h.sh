source tools/gpu_steps.sh
step r04_h_tests.log 400 python3 -u -m pytest tests/test_gpu_one_pass.py tests/test_gpu_edge.py tests/test_gpu_tile_costs.py -x -q --timeout 200 --timeout-method thread
step r04_h_ab.txt 900 bash tools/ab.sh "lib" 2 "head em8" RT_MEASURED_ORDER=1
cat gpurun_out/r04_h_ab.txt
step r04_h_ab_lds.txt 600 bash tools/ab.sh "lib" 2 "head em8" RT_LDS_STACK=13
cat gpurun_out/r04_h_ab_lds.txt
step r04_h_ab_base.txt 600 bash tools/ab.sh "lib" 2 "head em8"
cat gpurun_out/r04_h_ab_base.txt
step r04_h_exit_em8_nohelp.txt 200 env RT_DRAIN_HELP=0 RT_LIB_DIR=ray_tracying_amd/lib_exit python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --emulate 8 --emulate-rank 7
grep "rt exit" gpurun_out/r04_h_exit_em8_nohelp.txt
bash tools/measure_r04_shares.sh r04_hm measured 8 5
bash tools/measure_r04_shares.sh r04_hl lattice 8 5
