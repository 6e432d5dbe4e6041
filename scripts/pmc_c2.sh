# PMC passes (separate runs, counters only) of the checksum kernel on C2 and C2u
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for W in fixed4k c2u; do
  TAG=pmc_$W BENCH_ARGS="--workload $W" PMC_FILE=scripts/pmc_default.txt bash scripts/profile_pmc.sh || exit $?
done
