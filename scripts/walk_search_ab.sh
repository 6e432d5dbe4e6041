# A/B of the f3 search kernel shapes (diagnostic library, ZDBCRC_SEARCH_VARIANT)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-walk_ab}
mkdir -p $OUT
for v in ${VARIANTS:-0 1 2 3 4 5 0}; do
  ZDBCRC_LIB=0-db_amd/lib/libzdbcrc_diag.so ZDBCRC_SEARCH_VARIANT=$v timeout -k 10 200 \
    python3 scripts/walk_probe.py ${CHUNKS:-8388608} > $OUT/v$v.jsonl 2> $OUT/v$v.err || exit $?
  echo "{\"variant\": $v, \"res\": [$(paste -sd, $OUT/v$v.jsonl)]}" >> $OUT/ab.jsonl
done
