#!/bin/bash
# rocprofv3 evidence (kernel trace + FETCH/WRITE passes) for the C4 (2^25 x 100 B) and C3
# (Zipf R=4096) map sides with the current kernels
set -e
bash tools/gpu_prof.sh r02b_ts --record-bytes 100 --records 33554432 --partitions 1024
bash tools/gpu_prof.sh r02b_z4096 --dist zipf --partitions 4096
echo done > "$GRAFT_REPO_ROOT/gpurun_out/prof_c3c4_DONE"
