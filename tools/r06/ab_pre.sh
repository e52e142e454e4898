#!/bin/bash
# Round 6: parity of the fused sample + layout write, then alternating bench A/B of engine builds.
# usage: bash tools/r06/ab_pre.sh <tag> <lib>...   (lib "tree" = sparkucx_amd/libsgx.so)
tag=$1; shift
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_padded.py tests/test_streaming_commit.py tests/test_read_metrics.py \
  -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > "$out/pytest.log" 2>&1 || { tail -30 "$out/pytest.log"; exit 1; }
tail -2 "$out/pytest.log"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || exit $?
for rep in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = tree ]; then
      timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-live-pmc --steps 40 > "$out/bench_${lib}_$rep.log" 2>&1 || exit $?
    else
      timeout -k 10 200 python -u tools/ab_run.py tools/ab/libsgx_$lib.so bench --no-cpu-baseline --no-live-pmc --steps 40 > "$out/bench_${lib}_$rep.log" 2>&1 || exit $?
    fi
    grep '^{' "$out/bench_${lib}_$rep.log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$lib', $rep, j['value'], j['ms_per_step'], j['roofline']['frac'], j['roofline_map_side']['frac'], j['stages_ms_per_step'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- \
  python3 bench.py --steps 10 --no-cpu-baseline --no-live-pmc > "$out/bench_kt.log" 2>&1 || exit $?
echo done > "$out/DONE"
