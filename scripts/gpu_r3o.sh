#!/bin/bash
# OR filter: walk tests + C4 digest, search-rate probe, walk timing
set -o pipefail
mkdir -p gpurun_out/r3o
timeout -k 10 400 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu.py -k "walk or scan or c4" -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3o/pytest.log 2>&1 &&
timeout -k 10 300 python3 -u scripts/search_rate.py > gpurun_out/r3o/search_rate.jsonl 2> gpurun_out/r3o/search_rate.err &&
timeout -k 10 200 python3 -u scripts/walk_probe.py 8388608 4194304 > gpurun_out/r3o/walk_probe.jsonl 2>&1 &&
mkdir -p gpurun_out/r3n
timeout -k 10 400 python3 -u scripts/tool_timeline.py hip cpu > gpurun_out/r3n/timeline.jsonl 2> gpurun_out/r3n/timeline.err
