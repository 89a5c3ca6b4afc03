# r05: seven waves for whole frames (lib) against six (lib_prev); GPU parity suite on lib
source tools/gpu_steps.sh
step r05j_ab.txt 900 bash tools/ab.sh "lib lib_prev" 2 "head em8 c5 c2"
step r05j_c2_seven.txt 300 bash tools/ab.sh "lib" 1 "c2" RT_TRACE_SEVEN=1
step r05j_gpu_tests.log 1200 python3 -u -m pytest tests -m gpu -x -q --timeout 800 --timeout-method thread
