# r05: Markstein-quotient normalisation (rt_normalize3) in the shading kernels (one-pass
# shading, the logic step, the soft-shadow step): parity of the shading paths, then A/B
source tools/gpu_steps.sh
step r05t_parity.log 600 python3 -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_one_pass.py tests/test_gpu_configs.py tests/test_gpu_fused.py tests/test_gpu_parity.py
step r05t_ab.txt 600 bash tools/ab.sh "lib_prev lib" 2 "c3 c4 head em8"
