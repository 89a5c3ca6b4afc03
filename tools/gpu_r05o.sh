# r05: fp16 plane codes for planes-only scenes, perm-selected (lib_f16) vs address-selected
# (lib_f16a) code pairs, against the committed build (lib_prev) and this tree's default (lib)
source tools/gpu_steps.sh
RT_LIB_DIR=ray_tracying_amd/lib_f16a step r05o_f16a_parity.log 300 python3 -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_bench_calls.py::test_headline_frame_as_timed
step r05o_ab.txt 800 bash tools/ab.sh "lib_prev lib lib_f16 lib_f16a" 2 "head em8 c5 c3"
