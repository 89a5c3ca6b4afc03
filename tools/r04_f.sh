source tools/gpu_steps.sh
step r04_f_coop_tests.log 300 env RT_LIB_DIR=ray_tracying_amd/lib_coop python3 -u -m pytest tests/test_gpu_one_pass.py tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread
step r04_f_icull_tests.log 300 env RT_LIB_DIR=ray_tracying_amd/lib_icull python3 -u -m pytest tests/test_gpu_one_pass.py tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread
step r04_f_ab.txt 900 bash tools/ab.sh "lib lib_icull lib_coop lib_coop5" 1 "head em8 c2"
cat gpurun_out/r04_f_ab.txt
step r04_f_exit_em8.txt 200 env RT_LIB_DIR=ray_tracying_amd/lib_exit python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --emulate 8 --emulate-rank 7
grep "rt exit" gpurun_out/r04_f_exit_em8.txt
step r04_f_exit_head.txt 200 env RT_LIB_DIR=ray_tracying_amd/lib_exit python3 bench.py --no-cpu-baseline --steps 2 --warmup 1
grep "rt exit" gpurun_out/r04_f_exit_head.txt
step r04_f_gather.json 120 python3 tools/gather_cost.py gpurun_out/r04_f_gather_cost.json
cat gpurun_out/r04_f_gather_cost.json
step r04_f_c5.json 400 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --res 4096 --spp-sqrt 8
cat gpurun_out/r04_f_c5.json | tail -3
