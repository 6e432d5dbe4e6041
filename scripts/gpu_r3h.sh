#!/bin/bash
# f3 walk breakdown: per-chunk stamps of the fused walk (diagnostic library)
set -o pipefail
mkdir -p gpurun_out/r3i
export ZDBCRC_LIB=$PWD/0-db_amd/lib/libzdbcrc_diag.so
WALK_STAMPS_DUMP=gpurun_out/r3i timeout -k 10 300 python3 -u scripts/walk_stamps.py 8388608:0 16777216:0 16777216:2048 33554432:2048 > gpurun_out/r3i/stamps.jsonl 2> gpurun_out/r3i/stamps.err
