#!/bin/bash
# wider chunk searches (512 / 1024 threads) in the fused walk: A/B and stamps
set -o pipefail
mkdir -p gpurun_out/r3s
timeout -k 10 500 python3 -u scripts/walk_ab.py 2 8388608 base= nt512=ZDBCRC_SEARCH_NT:512 nt1024=ZDBCRC_SEARCH_NT:1024 > gpurun_out/r3s/ab8.jsonl 2> gpurun_out/r3s/ab.err &&
timeout -k 10 400 python3 -u scripts/walk_ab.py 2 4194304 base4= nt1024_4=ZDBCRC_SEARCH_NT:1024 > gpurun_out/r3s/ab4.jsonl 2>> gpurun_out/r3s/ab.err &&
ZDBCRC_SEARCH_NT=1024 ZDBCRC_LIB=$PWD/0-db_amd/lib/libzdbcrc_diag.so timeout -k 10 300 python3 -u scripts/walk_stamps.py 8388608:2048 4194304:2048 2097152:2048 > gpurun_out/r3s/stamps1024.jsonl 2>> gpurun_out/r3s/ab.err
