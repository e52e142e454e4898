set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/grp
timeout -k 10 600 python -u -m pytest tests/test_reduce_side.py tests/test_threads_streaming_combine.py tests/test_kryo.py tests/test_lz4.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/grp/pytest.log 2>&1 || { tail -40 gpurun_out/grp/pytest.log; exit 1; }
tail -1 gpurun_out/grp/pytest.log
bash tools/ab/r03_reduce_ab.sh grp "base tree"
