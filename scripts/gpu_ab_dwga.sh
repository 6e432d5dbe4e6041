# A/B: the dword grid for every record size with its fold dword loaded with the last superstep (DWGA)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r2e}
mkdir -p gpurun_out/$T
PROBE_BLOCKS=none timeout -k 10 400 python -u scripts/ab.py ${AB_WORK:-c2u,fixed4k,zipf} ${AB_VARIANTS:-31,32,0,33} > gpurun_out/$T/ab.jsonl 2> gpurun_out/$T/ab.err
