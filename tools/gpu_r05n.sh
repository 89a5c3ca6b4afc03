# r05: the issue class of v_fma_mix_f32; fp16 plane codes in 80-B device nodes (RT_NODE_F16=1,
# lib_f16: parity of the whole headline frame, then A/B); camera rays generated at refill
# (RT_CAM_IN_TRACE=1, lib_camtrace) vs camera_kernel + query record (lib)
source tools/gpu_steps.sh
step r05n_ubench_mix.txt 240 tools/bin/ubench_mix
RT_LIB_DIR=ray_tracying_amd/lib_f16 step r05n_f16_parity.log 400 python3 -u -m pytest -x -v --timeout 380 --timeout-method thread tests/test_gpu_bench_calls.py::test_headline_frame_as_timed tests/test_gpu_one_pass.py
RT_LIB_DIR=ray_tracying_amd/lib_camtrace step r05n_camtrace_parity.log 300 python3 -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_bench_calls.py::test_headline_frame_as_timed
step r05n_ab.txt 700 bash tools/ab.sh "lib lib_f16 lib_camtrace" 2 "head em8 c5 c3"
