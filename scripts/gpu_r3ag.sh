#!/bin/bash
# tail-pool parameters of the packed kernel at 1,024 threads (DYN / CPW / pools)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3ag
timeout -k 10 500 python -u scripts/ab.py c2u,fixed4k,zipf_le4096,zipf_le2048,c2u 68,76,77,78,79 > gpurun_out/r3ag/ab_packed_pools.jsonl 2> gpurun_out/r3ag/ab_packed_pools.err
