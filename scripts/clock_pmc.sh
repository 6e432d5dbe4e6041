# effective clock of the read probe and of the checksum kernel: GRBM_GUI_ACTIVE (sum over 8 XCDs) per dispatch
# next to the dispatch duration from the kernel trace of the same run
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-clock}
mkdir -p $OUT
PROBE_BLOCKS=${PROBE_BLOCKS:--104} timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace --output-format csv \
    -d $OUT/run -o clk -- python3 scripts/ab.py ${AB_WORK:-zipf} ${AB_VARIANTS:-0} > $OUT/ab.jsonl 2> $OUT/ab.err
