#!/bin/bash
# f3 walk with 16 MiB chunks for stores whose 8 MiB chunks outnumber the
# resident search workgroups: walk GPU tests, walk/scan times (default = 0,
# 8 MiB, 16 MiB), then the default bench line (C4 leg)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3y
timeout -k 10 400 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu.py -x -q -m gpu -k "walk or scan or c4 or store or check" --timeout 120 --timeout-method thread > gpurun_out/r3y/pytest_walk.log 2>&1 &&
timeout -k 10 240 python -u scripts/walk_probe.py 0 8388608 16777216 0 > gpurun_out/r3y/walk_probe.jsonl 2> gpurun_out/r3y/walk_probe.err &&
timeout -k 10 400 python -u bench.py > gpurun_out/r3y/bench.json 2> gpurun_out/r3y/bench.err
