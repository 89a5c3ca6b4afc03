source tools/gpu_steps.sh
step r04_c_onepass.log 300 python3 -u -m pytest tests/test_gpu_one_pass.py -x -q --timeout 120 --timeout-method thread
step r04_c_ab.txt 900 bash tools/ab.sh "lib_base lib lib_sr64 lib_sr64w8" 1 "head em8 c3"
cat gpurun_out/r04_c_ab.txt
