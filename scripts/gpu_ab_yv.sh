# GPU tests, then the dword-grid kernel (fold dword prefetched at segment setup)
# against the round-2 HEAD kernels (a diagnostic build of the previous commit)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r2c_yv}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1 && \
PROBE_BLOCKS=none timeout -k 10 400 python -u scripts/ab.py zipf,c2u,fixed4k 0,30,26,31 > gpurun_out/$T/ab.jsonl 2> gpurun_out/$T/ab.err && \
ZDBCRC_LIB=0-db_amd/lib/libzdbcrc_diag_head.so PROBE_BLOCKS=none timeout -k 10 300 python -u scripts/ab.py zipf,c2u,fixed4k 0,26 > gpurun_out/$T/ab_head.jsonl 2> gpurun_out/$T/ab_head.err
