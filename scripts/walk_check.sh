# f3 walk GPU tests (product library) and the walk timing on the C4 shard
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-walk_check}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_walk.py tests/test_c4.py tests/test_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 && \
timeout -k 10 200 python3 scripts/walk_probe.py 8388608 > $OUT/probe.jsonl 2> $OUT/probe.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 scripts/walk_probe.py 8388608 > $OUT/probe_traced.jsonl 2> $OUT/probe_traced.err
