# round-2 resume: GPU tests (product library), then the dword-grid A/B and the f3 walk A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r2c}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1 && \
PROBE_BLOCKS=none timeout -k 10 400 python -u scripts/ab.py ${AB_WORK:-c2u,fixed4k,zipf} ${AB_VARIANTS:-0,30,26,31} > gpurun_out/$T/ab.jsonl 2> gpurun_out/$T/ab.err && \
TAG=$T/walk bash scripts/walk_ab2.sh
