source tools/gpu_steps.sh
step r04_a_onepass.log 300 python3 -u -m pytest tests/test_gpu_one_pass.py -x -v --timeout 120 --timeout-method thread
step r04_a_gpu.log 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step r04_a_ab.txt 600 bash tools/ab.sh "lib_base lib" 1 "head em8 c2 c3"
cat gpurun_out/r04_a_ab.txt
