#!/bin/bash
# small-record store walk per chunk size (and the density default), walk tests; tool exit-cost timeline
set -o pipefail
mkdir -p gpurun_out/r3q
timeout -k 10 400 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu.py -k "walk or scan or c4" -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3q/pytest.log 2>&1 &&
timeout -k 10 300 python3 -u scripts/walk_small_records.py 4096 > gpurun_out/r3q/small_records.jsonl 2> gpurun_out/r3q/small_records.err &&
timeout -k 10 200 python3 -u scripts/walk_probe.py 0 8388608 > gpurun_out/r3q/walk_probe.jsonl 2>&1 &&
timeout -k 10 500 python3 -u scripts/tool_timeline.py hip > gpurun_out/r3q/timeline.jsonl 2> gpurun_out/r3q/timeline.err
