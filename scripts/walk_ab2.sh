# f3 A/B: search occupancy variants x chain shape (diagnostic library);
# first the GPU walk tests with the windowed chain (correctness), then timings
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-walk_ab2}
mkdir -p $OUT
export ZDBCRC_LIB=0-db_amd/lib/libzdbcrc_diag.so
ZDBCRC_CHAIN_MODE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_walk.py -x -q -m gpu --timeout 120 \
    --timeout-method thread > $OUT/pytest_walk_win.log 2>&1 || exit $?
for cfg in ${CONFIGS:-"0 0" "0 1" "11 0" "11 1" "12 1" "10 1" "0 0" "0 1"}; do
  set -- $cfg
  ZDBCRC_SEARCH_VARIANT=$1 ZDBCRC_CHAIN_MODE=$2 timeout -k 10 200 \
    python3 scripts/walk_probe.py ${CHUNKS:-8388608 16777216 4194304} > $OUT/s$1_c$2.jsonl 2> $OUT/s$1_c$2.err || exit $?
  echo "{\"search_variant\": $1, \"chain_mode\": $2, \"res\": [$(paste -sd, $OUT/s$1_c$2.jsonl)]}" >> $OUT/ab.jsonl
done
