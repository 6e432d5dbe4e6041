#!/bin/bash
# packed kernel (one load buffer, 768 threads) for every bounded batch <= 4 KiB: smoke, full GPU suite, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3ad
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3ad/smoke.log 2>&1 &&
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3ad/pytest_gpu.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/r3ad/bench.json 2> gpurun_out/r3ad/bench.err
