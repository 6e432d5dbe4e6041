#!/bin/bash
# product packed kernels in rows of 16 / 8 / 4 lanes: full GPU suite + smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3z
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3z/smoke.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3z/pytest_gpu.log 2>&1
