# r05: XCD-aware deal of the work queue (RT_XCD_CHUNK groups per chunk, chunks dealt to the
# shards of one XCD): parity of the whole headline frame, then a sweep
source tools/gpu_steps.sh
RT_XCD_CHUNK=64 step r05v_parity.log 300 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_bench_calls.py::test_headline_frame_as_timed
step r05v_x0.txt 300 bash tools/ab.sh lib 2 "head em8 c5"
step r05v_x64.txt 300 bash tools/ab.sh lib 2 "head em8 c5" RT_XCD_CHUNK=64
step r05v_x512.txt 300 bash tools/ab.sh lib 2 "head em8 c5" RT_XCD_CHUNK=512
step r05v_x6400.txt 300 bash tools/ab.sh lib 2 "head em8 c5" RT_XCD_CHUNK=6400
