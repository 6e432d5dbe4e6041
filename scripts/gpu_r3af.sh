#!/bin/bash
# loads of the line shared across a superstep boundary without the nontemporal
# hint (TEL): packed kernel on C2u / C2 / Zipf <= 4 KiB, main kernel on C3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3af
timeout -k 10 420 python -u scripts/ab.py c2u,fixed4k,zipf_le4096,c2u 68,71,72,69,73 > gpurun_out/r3af/ab_tel_packed.jsonl 2> gpurun_out/r3af/ab_tel_packed.err &&
timeout -k 10 300 python -u scripts/ab.py zipf,zipf 0,75 > gpurun_out/r3af/ab_tel_main.jsonl 2> gpurun_out/r3af/ab_tel_main.err
