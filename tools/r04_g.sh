source tools/gpu_steps.sh
step r04_g_tests.log 400 python3 -u -m pytest tests/test_gpu_one_pass.py tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_edge.py -x -q --timeout 200 --timeout-method thread
step r04_g_exit_em8.txt 200 env RT_LIB_DIR=ray_tracying_amd/lib_exit python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --emulate 8 --emulate-rank 7
grep "rt exit" gpurun_out/r04_g_exit_em8.txt
step r04_g_exit_em8e.txt 200 env RT_MEASURED_ORDER=0 RT_LIB_DIR=ray_tracying_amd/lib_exit python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --emulate 8 --emulate-rank 7
grep "rt exit" gpurun_out/r04_g_exit_em8e.txt
step r04_g_ab.txt 900 bash tools/ab.sh "lib_prev lib" 2 "head em8 em4"
cat gpurun_out/r04_g_ab.txt
step r04_g_ab_est.txt 600 bash tools/ab.sh "lib" 2 "head em8 em4" RT_MEASURED_ORDER=0
cat gpurun_out/r04_g_ab_est.txt
