# GPU tests, dword-grid threshold A/B, bench (product library)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r2d}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1 && \
PROBE_BLOCKS=none timeout -k 10 400 python -u scripts/ab.py zipf,c2u,fixed4k 0,30,26,31 > gpurun_out/$T/ab.jsonl 2> gpurun_out/$T/ab.err && \
timeout -k 10 600 python bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
