#!/bin/bash
# Write-combining 100 B K4 in the reduce side's digit / key-window passes (libsgx_wwcred.so:
# -DSGX_WIDE_WC_REDUCE=1) against the default: reduce-side GPU tests on the variant, then
# tools/prof_reduce.py sorted:terasort alternated.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04zr
timeout -k 10 700 python -u -c "
import sys, sparkucx_amd._lib as L, pytest
L.LIB_PATH = 'tools/ab/libsgx_wwcred.so'
sys.exit(pytest.main(['-x', '-q', '--timeout', '200', '--timeout-method', 'thread', '-m', 'gpu',
    'tests/test_reduce_side.py', 'tests/test_gpu_parity.py', 'tests/test_exchange_multirank.py', '-k', 'sort or terasort or TeraSort or wide or range or exchange']))
" > gpurun_out/r04zr/pytest_wwcred.log 2>&1 || { tail -40 gpurun_out/r04zr/pytest_wwcred.log; exit 1; }
tail -1 gpurun_out/r04zr/pytest_wwcred.log
for i in 1 2; do
  timeout -k 10 240 python -u tools/prof_reduce.py --cases sorted:terasort --iters 5 > gpurun_out/r04zr/default_$i.log 2>&1 || exit 1
  timeout -k 10 240 python -u tools/ab_run.py tools/ab/libsgx_wwcred.so prof_reduce --cases sorted:terasort --iters 5 > gpurun_out/r04zr/wwcred_$i.log 2>&1 || exit 1
done
grep -h '^{' gpurun_out/r04zr/*_?.log | cut -c1-300
