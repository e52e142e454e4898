#!/bin/bash
# k_scatter_wide_wc phase stamps (finer merge split).
tag=${1:-r05l}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "$1"; tail -40 "$2"; exit 1; }
for v in ${VARIANTS:-stamps}; do
  timeout -k 10 180 python -u tools/ab_run.py tools/ab/libsgx_$v.so wc_stamps --record-bytes 100 --wide-wc $STAMP_ARGS > "$out/$v.log" 2>&1 || fail "stamps $v" "$out/$v.log"
  tail -1 "$out/$v.log"
done
echo done > "$out/DONE"
