# A/B of chains per wave in the f3 chain kernels (diagnostic library)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-walk_chain_ab}
mkdir -p $OUT
for c in ${CPWS:-16 8 4 2 32 16}; do
  ZDBCRC_LIB=0-db_amd/lib/libzdbcrc_diag.so ZDBCRC_CHAINS_PER_WAVE=$c timeout -k 10 200 \
    python3 scripts/walk_probe.py ${CHUNK:-8388608} 2097152 > $OUT/c$c.jsonl 2> $OUT/c$c.err || exit $?
  echo "{\"chains_per_wave\": $c, \"res\": [$(paste -sd, $OUT/c$c.jsonl)]}" >> $OUT/ab.jsonl
done
