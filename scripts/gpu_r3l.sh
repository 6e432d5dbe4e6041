#!/bin/bash
# skewed chunk edges: walk tests on the diagnostic library with the skew, then A/B
set -o pipefail
mkdir -p gpurun_out/r3l
ZDBCRC_LIB=$PWD/0-db_amd/lib/libzdbcrc_diag.so ZDBCRC_CHUNK_SKEW=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_walk.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3l/pytest_skew.log 2>&1 &&
timeout -k 10 500 python3 -u scripts/walk_ab.py 3 8388608 base= skew=ZDBCRC_CHUNK_SKEW:1 > gpurun_out/r3l/ab.jsonl 2> gpurun_out/r3l/ab.err &&
timeout -k 10 300 python3 -u scripts/walk_ab.py 2 16777216 base16= skew16=ZDBCRC_CHUNK_SKEW:1 >> gpurun_out/r3l/ab.jsonl 2>> gpurun_out/r3l/ab.err
