# r05 A/B: the soft-light instance over transformed shapes at 5 waves (lib_soft5, C4), the fused
# transformed instance at 6 (lib_fuse6, C3) against lib
source tools/gpu_steps.sh
step r05k_ab.txt 900 bash tools/ab.sh "lib lib_soft5 lib_fuse6" 2 "c4 c3"
