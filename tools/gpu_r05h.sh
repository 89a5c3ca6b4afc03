# r05: reflection chains in the tracing lane (kRefl): parity tests, then C4 with and without
source tools/gpu_steps.sh
step r05h_tests.log 900 python3 -u -m pytest tests/test_gpu_fused.py tests/test_gpu_configs.py tests/test_gpu_knobs.py -x -v --timeout 600 --timeout-method thread
step r05h_c4_refl.txt 600 bash tools/ab.sh "lib" 2 "c4" RT_REFL_FUSE=1
step r05h_c4_norefl.txt 600 bash tools/ab.sh "lib" 2 "c4" RT_REFL_FUSE=0
