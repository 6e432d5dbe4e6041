#!/bin/bash
# product tree check: full GPU suite, then the default bench line
set -o pipefail
mkdir -p gpurun_out/r3m
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3m/pytest_gpu.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r3m/bench.json 2> gpurun_out/r3m/bench.err
