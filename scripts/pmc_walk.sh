# PMC passes over the f3 walk kernels (scripts/walk_probe.py, one chunk size)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc_walk}
mkdir -p $OUT
i=0
while IFS= read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $counters --kernel-include-regex walk_ --output-format csv \
      -d $OUT/pass$i -o pmc -- python3 scripts/walk_probe.py ${CHUNK:-8388608} > $OUT/pass$i.json 2> $OUT/pass$i.err || { rc=$?; echo "pass $i failed rc=$rc" >> $OUT/status; [ $rc -ge 124 ] && exit $rc; }
done < ${PMC_FILE:-scripts/pmc_walk.txt}
echo done >> $OUT/status
