source tools/gpu_steps.sh
step r04_e_exit_em8.txt 200 env RT_LIB_DIR=ray_tracying_amd/lib_exit python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --emulate 8 --emulate-rank 7
grep "rt exit" gpurun_out/r04_e_exit_em8.txt
step r04_e_exit_head.txt 200 env RT_LIB_DIR=ray_tracying_amd/lib_exit python3 bench.py --no-cpu-baseline --steps 2 --warmup 1
grep "rt exit" gpurun_out/r04_e_exit_head.txt
step r04_e_exit_c2.txt 200 env RT_LIB_DIR=ray_tracying_amd/lib_exit python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --primary-only --spp-sqrt 1
grep "rt exit" gpurun_out/r04_e_exit_c2.txt
step r04_e_c5.json 400 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --res 4096 --spp-sqrt 8
cat gpurun_out/r04_e_c5.json | tail -3
step r04_e_gather.json 120 python3 tools/gather_cost.py gpurun_out/r04_e_gather_cost.json
cat gpurun_out/r04_e_gather_cost.json
step r04_e_ab.txt 900 bash tools/ab.sh "lib lib_icull" 2 "head em8 c2 c3"
cat gpurun_out/r04_e_ab.txt
