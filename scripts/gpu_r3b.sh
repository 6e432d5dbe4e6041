# packed small-record kernel: correctness on crafted batches, then A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r3b}
mkdir -p gpurun_out/$T
timeout -k 10 300 python scripts/pk_check.py 42,44,46 > gpurun_out/$T/pk_check.jsonl 2> gpurun_out/$T/pk_check.err && \
PROBE_MIB= timeout -k 10 500 python scripts/ab.py c2u,fixed4k,zipf_small 33,42,44,46 > gpurun_out/$T/ab_pk.jsonl 2> gpurun_out/$T/ab_pk.err
