# kernel trace + stats of the bench (rocprofv3), plus the counter list
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-prof}
mkdir -p $OUT
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err
