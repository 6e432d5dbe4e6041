#!/bin/bash
# the main kernel at 1,024 threads (64 VGPRs, 8 waves per SIMD) against 768 on C3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3ah
timeout -k 10 300 python -u scripts/ab.py zipf,zipf,zipf 0,80 > gpurun_out/r3ah/ab_main_1024.jsonl 2> gpurun_out/r3ah/ab_main_1024.err
