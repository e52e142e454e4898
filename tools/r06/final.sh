#!/bin/bash
# Round 6, last validation of the final tree: part A (GPU suite, smoke, bench lines), then the
# C3 PMC / kernel profile again (its tail changed after part C ran).
tag=${1:-r06f}
bash tools/r06/validate.sh $tag || exit $?
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_prof.sh $tag/prof_c3 --partitions 4096 --dist zipf || exit 1
echo done > "$out/DONE2"
