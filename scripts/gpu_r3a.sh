# round 3 start: GPU tests on the round-2 tree + per-class cost split of C3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r3a}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1 && \
PROBE_MIB= timeout -k 10 400 python scripts/ab.py zipf,zipf_small,zipf_large,c2u,fixed4k 0,33 > gpurun_out/$T/ab_split.jsonl 2> gpurun_out/$T/ab_split.err
