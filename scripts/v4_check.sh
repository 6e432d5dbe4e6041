#!/bin/bash
# v4 bring-up: A/B against v3 (bit-exact vs variant listed first), per-wave stamps, GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 scripts/ab.py zipf,fixed4k,single ${AB_VARIANTS:-2,0,6} > gpurun_out/ab16.jsonl 2>&1 &&
timeout -k 10 300 python3 scripts/stamps.py zipf v4_wg768_stamp > gpurun_out/stamps6.txt 2>&1 &&
timeout -k 10 300 python3 scripts/stamps.py zipf v3_wg768_prio_stamp >> gpurun_out/stamps6.txt 2>&1 &&
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_v4.txt 2>&1
