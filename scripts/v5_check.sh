#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 scripts/ab.py zipf,fixed4k,single ${AB_VARIANTS:-0,1,2,3,7} > gpurun_out/ab17.jsonl 2>&1 &&
timeout -k 10 300 python3 scripts/stamps.py zipf v5_wg1024_prio_stamp > gpurun_out/stamps7.txt 2>&1 &&
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_v5.txt 2>&1
