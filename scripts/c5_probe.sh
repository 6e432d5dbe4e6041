# C5 latency probe on the GPU box: plain run (the diagnostic library also
# A/Bs how results come back), then the product library under a kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-c5}
mkdir -p gpurun_out/$T
gcc -O2 -o /tmp/c5_probe scripts/c5_probe.c -ldl && \
timeout -k 10 120 /tmp/c5_probe ${C5_LIB:-0-db_amd/lib/libzdbcrc.so} > gpurun_out/$T/c5_probe.jsonl 2>&1 && \
if [ -n "$C5_TRACE" ]; then
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o c5 -- /tmp/c5_probe > gpurun_out/$T/c5_probe_traced.jsonl 2>&1
fi
