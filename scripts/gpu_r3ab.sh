#!/bin/bash
# new at-scale packed-shape tests, then the two-rank rehearsal of bench.py on one GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3ab
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v -m gpu -k "packed" --timeout 200 --timeout-method thread > gpurun_out/r3ab/pytest_packed.log 2>&1 &&
timeout -k 10 600 python -u bench.py --gpus 2 --rehearsal --steps 10 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/r3ab/bench_n2_rehearsal.json 2> gpurun_out/r3ab/bench_n2_rehearsal.err
