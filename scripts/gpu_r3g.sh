#!/bin/bash
# chain-window A/B on the C4 shard (diagnostic library)
set -o pipefail
mkdir -p gpurun_out/r3g
timeout -k 10 400 python -u scripts/walk_wb.py 0 1024 2048 4096 8192 > gpurun_out/r3g/walk_wb.jsonl 2> gpurun_out/r3g/walk_wb.err
