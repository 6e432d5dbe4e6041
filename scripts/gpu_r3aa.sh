#!/bin/bash
# split batches (small records to the packed kernel): full GPU suite + smoke,
# A/B of the split threshold on C3 / C2 / C2u (unbounded calls), bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3aa
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3aa/smoke.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3aa/pytest_gpu.log 2>&1 &&
PROBE_BLOCKS=none timeout -k 10 500 python -u scripts/ab.py zipf,fixed4k,c2u,zipf 0,0s256,0s1024,0s2048 > gpurun_out/r3aa/ab_split.jsonl 2> gpurun_out/r3aa/ab_split.err &&
timeout -k 10 400 python -u bench.py > gpurun_out/r3aa/bench.json 2> gpurun_out/r3aa/bench.err
