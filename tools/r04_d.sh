source tools/gpu_steps.sh
step r04_d_ubench_mix.txt 200 tools/bin/ubench_mix
cat gpurun_out/r04_d_ubench_mix.txt
step r04_d_onepass.log 300 python3 -u -m pytest tests/test_gpu_one_pass.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread
step r04_d_ab.txt 900 bash tools/ab.sh "lib_prev lib lib_icull" 1 "head em8 c3 c2"
cat gpurun_out/r04_d_ab.txt
