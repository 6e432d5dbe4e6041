# PMC passes (rocprofv3 --pmc, one counter group per pass, no other tracing)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc}
mkdir -p $OUT
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-extra ${BENCH_ARGS}"
i=0
while IFS= read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $counters --kernel-include-regex ${KREGEX:-crc_batch_kernel} --output-format csv \
      -d $OUT/pass$i -o pmc -- python3 bench.py $ARGS > $OUT/pass$i.json 2> $OUT/pass$i.err || { rc=$?; echo "pass $i failed rc=$rc" >> $OUT/status; [ $rc -ge 124 ] && exit $rc; }
done < ${PMC_FILE:-scripts/pmc_default.txt}
echo done >> $OUT/status
