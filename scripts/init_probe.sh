# GPU engine start-up on a fresh box: the HIP runtime calls one by one
# (hip_init_breakdown.cpp), then the integrity tool's own trace on a 256 MiB
# reference-written datafile, GPU and auto engines (each run a fresh process)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-init}
mkdir -p gpurun_out/$T
hipcc -O2 --offload-arch=gfx950 -Wno-unused-value scripts/hip_init_breakdown.cpp -ldl -o /tmp/hib
for i in 1 2 3; do
    timeout -k 10 60 /tmp/hib 0-db_amd/lib/libzdbcrc.so >> gpurun_out/$T/breakdown.jsonl || exit 1
done
D=/tmp/init_df
rm -rf $D && mkdir -p $D
oracle/_ref/gen_datafile_ref $D fixed 65000 99 4096 > /dev/null 2>&1
ln -s d0 $D/data/default/zdb-data-0
for e in hip hip hip auto; do
    ( time -p env ZDBCRC_TOOL_TRACE=1 TZ=UTC timeout -k 10 60 0-db_amd/bin/zdb-integrity-check --engine=$e \
        $D/data/default/zdb-data-0 > /dev/null ) 2>&1 | grep -E "^\[trace\]|^real" >> gpurun_out/$T/tool_trace.txt
done
