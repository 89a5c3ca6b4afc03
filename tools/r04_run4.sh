set -e
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r04_n2_tests.log 2>&1
tail -n 2 gpurun_out/r04_n2_tests.log
bash tools/ab.sh "lib lib_prev" 2 "head em8 c5 c3"
