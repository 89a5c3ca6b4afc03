# r05: kRefl parity + C4 A/B; node-visit A/Bs (cull keys by shifts, bf16 nodes, both); seven waves
source tools/gpu_steps.sh
step r05h_tests.log 900 python3 -u -m pytest tests/test_gpu_fused.py tests/test_gpu_configs.py tests/test_gpu_knobs.py -x -v --timeout 600 --timeout-method thread
step r05h_c4.txt 600 bash tools/ab.sh "lib" 2 "c4" RT_REFL_FUSE=1
step r05h_c4_norefl.txt 600 bash tools/ab.sh "lib" 2 "c4" RT_REFL_FUSE=0
step r05g_ab.txt 900 bash tools/ab.sh "lib lib_cmask lib_bf16 lib_bfcm" 2 "head em8 c5"
step r05g_w7.txt 300 bash tools/ab.sh "lib_w7" 1 "head em8 c5" RT_LDS_STACK=11
