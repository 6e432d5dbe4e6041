#!/bin/bash
# packed kernel in the product (records <= 2 KiB): full GPU suite
set -o pipefail
mkdir -p gpurun_out/r3u
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3u/pytest_gpu.log 2>&1
