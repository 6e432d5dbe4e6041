#!/bin/bash
# resumed round 3: full GPU suite with the vector-metadata packed kernel, then
# the read probes of the packed access shapes (rows of 4 / 8 / 16 / 64 lanes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3w
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3w/pytest_gpu.log 2>&1 &&
PROBE_BLOCKS=-104,-304,-344,-308,-316,-364,-104 timeout -k 10 300 python -u scripts/ab.py none > gpurun_out/r3w/probe.jsonl 2> gpurun_out/r3w/probe.err
