source tools/gpu_steps.sh
step r04_h_tests.log 400 python3 -u -m pytest tests/test_gpu_one_pass.py tests/test_gpu_edge.py tests/test_gpu_tile_costs.py tests/test_bench_ranks.py -x -q --timeout 200 --timeout-method thread
step r04_h_ab_base.txt 600 bash tools/ab.sh "lib" 2 "head em8"
cat gpurun_out/r04_h_ab_base.txt
export BENCH_EXTRA="--frames-in-flight 2"
step r04_h_ab_f2.txt 600 bash tools/ab.sh "lib" 2 "head em8 em4 c3"
cat gpurun_out/r04_h_ab_f2.txt
unset BENCH_EXTRA
step r04_h_ab_lds.txt 600 bash tools/ab.sh "lib" 2 "head em8" RT_LDS_STACK=13
cat gpurun_out/r04_h_ab_lds.txt
step r04_h_ab_dl.txt 600 bash tools/ab.sh "lib" 2 "head em8" RT_DRAIN_LEAF_DIV=2
cat gpurun_out/r04_h_ab_dl.txt
step r04_h_ab_mo.txt 600 bash tools/ab.sh "lib" 1 "head em8" RT_MEASURED_ORDER=1
cat gpurun_out/r04_h_ab_mo.txt
