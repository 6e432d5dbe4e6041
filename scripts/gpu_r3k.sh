#!/bin/bash
# search filter A/B (two-pass ILP vs per-row), walk tests with the ILP variant
set -o pipefail
mkdir -p gpurun_out/r3k
timeout -k 10 500 python3 -u scripts/walk_ab.py 3 8388608 base= ilp=ZDBCRC_SEARCH_ILP:1 ilp_mw5=ZDBCRC_SEARCH_ILP:1,ZDBCRC_SEARCH_ILP_MW:5 > gpurun_out/r3k/ab.jsonl 2> gpurun_out/r3k/ab.err
