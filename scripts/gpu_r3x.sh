#!/bin/bash
# f3 walk: search width (threads per chunk) x chunk size on the C4 shard --
# walk and scan times (walk_probe.py), per-chunk stamps (walk_stamps.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export ZDBCRC_LIB=$GRAFT_REPO_ROOT/0-db_amd/lib/libzdbcrc_diag.so
mkdir -p gpurun_out/r3x
for NT in 256 384 512; do
  ZDBCRC_SEARCH_NT=$NT timeout -k 10 240 python -u scripts/walk_probe.py 8388608 16777216 > gpurun_out/r3x/probe_nt$NT.jsonl 2> gpurun_out/r3x/probe_nt$NT.err || exit $?
done
for NT in 256 384; do
  ZDBCRC_SEARCH_NT=$NT timeout -k 10 240 python -u scripts/walk_stamps.py 8388608:2048 16777216:2048 > gpurun_out/r3x/stamps_nt$NT.jsonl 2> gpurun_out/r3x/stamps_nt$NT.err || exit $?
done
