#!/bin/bash
# wave stitch: walk tests + C4 digest; walk timing; kernel trace; PMC passes on the split search
set -o pipefail
mkdir -p gpurun_out/r3j
timeout -k 10 400 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu.py -k "walk or scan or c4" -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3j/pytest.log 2>&1 &&
timeout -k 10 200 python3 -u scripts/walk_probe.py 8388608 16777216 > gpurun_out/r3j/walk_probe.jsonl 2>&1 &&
ZDBCRC_LIB=$PWD/0-db_amd/lib/libzdbcrc_diag.so ZDBCRC_SERIAL_STITCH=1 timeout -k 10 200 python3 -u scripts/walk_probe.py 8388608 16777216 > gpurun_out/r3j/walk_probe_serial_stitch.jsonl 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3j/kt -o run -- python3 -u scripts/walk_probe.py 8388608 > gpurun_out/r3j/kt.log 2>&1 &&
ZDBCRC_LIB=$PWD/0-db_amd/lib/libzdbcrc_diag.so ZDBCRC_CHAIN_MODE=1 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU -d gpurun_out/r3j/p1 -o run --output-format csv -- python3 -u scripts/walk_probe.py 8388608 > gpurun_out/r3j/p1.log 2>&1 &&
ZDBCRC_LIB=$PWD/0-db_amd/lib/libzdbcrc_diag.so ZDBCRC_CHAIN_MODE=1 timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_IFETCH SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA -d gpurun_out/r3j/p2 -o run --output-format csv -- python3 -u scripts/walk_probe.py 8388608 > gpurun_out/r3j/p2.log 2>&1
