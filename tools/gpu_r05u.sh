# r05: sort keys with LDS-parked child entries in the node visit (RT_KEY_SORT=1, lib_ks):
# parity of the whole headline frame and the one-pass paths, then A/B
source tools/gpu_steps.sh
RT_LIB_DIR=ray_tracying_amd/lib_ks step r05u_parity.log 500 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_bench_calls.py::test_headline_frame_as_timed tests/test_gpu_one_pass.py tests/test_gpu_scale.py
step r05u_ab.txt 600 bash tools/ab.sh "lib lib_ks" 2 "head em8 c5 c2"
