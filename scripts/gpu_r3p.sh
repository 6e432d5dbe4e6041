#!/bin/bash
# f1: tool GPU tests, then the ingest timeline (pinned vs staged)
set -o pipefail
mkdir -p gpurun_out/r3p
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -k "tool" -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3p/pytest.log 2>&1 &&
timeout -k 10 500 python3 -u scripts/tool_timeline.py hip cpu > gpurun_out/r3p/timeline.jsonl 2> gpurun_out/r3p/timeline.err
