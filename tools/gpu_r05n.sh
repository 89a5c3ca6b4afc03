# r05: camera rays generated at refill (RT_CAM_IN_TRACE=1, lib_camtrace)
# vs camera_kernel + query record (lib); then the SAH build-parameter sweep
source tools/gpu_steps.sh
step r05n_ab_camtrace.txt 600 bash tools/ab.sh "lib lib_camtrace" 2 "head em8 c5 c3"
step r05m_node025.txt 200 bash tools/ab.sh "lib" 1 "head em8" RT_SAH_NODE=0.25
step r05m_node1.txt 200 bash tools/ab.sh "lib" 1 "head em8" RT_SAH_NODE=1.0
step r05m_leaf2.txt 200 bash tools/ab.sh "lib" 1 "head em8" RT_SAH_LEAF=2
step r05m_leaf6.txt 200 bash tools/ab.sh "lib" 1 "head em8" RT_SAH_LEAF=6
