# PMC passes (separate runs, counters only) of the checksum kernel on C2 and C2u (max_length 4096: the packed kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for W in fixed4k c2u; do
  TAG=pmc_$W KREGEX=crc_packed_kernel BENCH_ARGS="--workload $W" PMC_FILE=scripts/pmc_default.txt bash scripts/profile_pmc.sh || exit $?
done
