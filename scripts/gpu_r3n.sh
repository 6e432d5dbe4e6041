#!/bin/bash
# f1 ingest timeline of the integrity-check tool
set -o pipefail
mkdir -p gpurun_out/r3n
timeout -k 10 400 python3 -u scripts/tool_timeline.py > gpurun_out/r3n/timeline.jsonl 2> gpurun_out/r3n/timeline.err
