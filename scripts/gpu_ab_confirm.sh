# GPU walk tests on the product library (windowed chain default), then a
# second-box confirmation of the dword-grid A/B (reversed order)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r2c_confirm}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_walk.py tests/test_c4.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_walk.log 2>&1 && \
PROBE_BLOCKS=none timeout -k 10 400 python -u scripts/ab.py ${AB_WORK:-zipf,c2u,fixed4k} ${AB_VARIANTS:-30,0,31,26} > gpurun_out/$T/ab.jsonl 2> gpurun_out/$T/ab.err
