# f3: the windowed chain fused into the search kernel (chain mode 2) vs separate kernels (1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-walk_ab3}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_walk.py tests/test_c4.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_walk_product.log 2>&1 || exit $?
export ZDBCRC_LIB=0-db_amd/lib/libzdbcrc_diag.so
ZDBCRC_CHAIN_MODE=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_walk.py tests/test_c4.py -x -q -m gpu --timeout 120 \
    --timeout-method thread > $OUT/pytest_walk_fused.log 2>&1 || exit $?
for cfg in ${CONFIGS:-"0 1" "0 2" "0 1" "0 2"}; do
  set -- $cfg
  ZDBCRC_SEARCH_VARIANT=$1 ZDBCRC_CHAIN_MODE=$2 timeout -k 10 200 \
    python3 scripts/walk_probe.py ${CHUNKS:-8388608 4194304 16777216} > $OUT/s$1_c$2.jsonl 2> $OUT/s$1_c$2.err || exit $?
  echo "{\"search_variant\": $1, \"chain_mode\": $2, \"res\": [$(paste -sd, $OUT/s$1_c$2.jsonl)]}" >> $OUT/ab.jsonl
done
