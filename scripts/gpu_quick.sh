# GPU tests, then a bench run (each step under its own time limit, chained with &&)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-quick}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} ${PYTEST_ARGS} > gpurun_out/$T/pytest_gpu.log 2>&1 && \
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
