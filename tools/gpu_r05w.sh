# r05: XCD-aware deal at 64 groups per chunk (lib_x64) vs the round-robin deal (lib), interleaved
source tools/gpu_steps.sh
step r05w_ab.txt 600 bash tools/ab.sh "lib lib_x64" 3 "head em8 c5"
