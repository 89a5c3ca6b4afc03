source tools/gpu_steps.sh
step r05e_ubench_mix.txt 300 tools/bin/ubench_mix
step r05e_gpu_tests.log 1200 python3 -u -m pytest tests -m gpu -x -q --timeout 800 --timeout-method thread
