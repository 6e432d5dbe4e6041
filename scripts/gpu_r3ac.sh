#!/bin/bash
# PMC passes on C2 / C2u (the small-record shape), then a kernel trace of the
# packed shapes (rows of 16 / 8 / 4) on small-record workloads
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3ac
for W in fixed4k c2u; do
  TAG=r3ac/pmc_$W BENCH_ARGS="--workload $W --no-c4" PMC_FILE=scripts/pmc_default.txt bash scripts/profile_pmc.sh || exit $?
done
PROBE_BLOCKS=none SETTLE_S=0.3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3ac/pk_trace -o run -- \
    python3 scripts/ab.py fixed2048,zipf_le1024@2048,zipf_le256@1024 49,56,57 > gpurun_out/r3ac/pk_ab.jsonl 2> gpurun_out/r3ac/pk_ab.err
