#!/bin/bash
# rows of 32 lanes vs 16 on 4 KiB records (A/B), then smoke, full GPU suite, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3ae
PROBE_BLOCKS=none timeout -k 10 400 python -u scripts/ab.py fixed4k,c2u,zipf_le4096,c2u 60,64,61 > gpurun_out/r3ae/ab_rw32.jsonl 2> gpurun_out/r3ae/ab_rw32.err &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3ae/smoke.log 2>&1 &&
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3ae/pytest_gpu.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/r3ae/bench.json 2> gpurun_out/r3ae/bench.err
