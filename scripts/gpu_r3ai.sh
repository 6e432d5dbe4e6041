#!/bin/bash
# C2u / C2 kernel time by where the leg runs: as the main leg, as an extra leg
# without the C4 leg before it (bench's full run has C4's 17 GB images first)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3ai
timeout -k 10 300 python bench.py --workload c2u --no-extra --no-cpu-baseline > gpurun_out/r3ai/c2u_main.json 2> gpurun_out/r3ai/c2u_main.err &&
timeout -k 10 400 python bench.py --no-c4 --no-cpu-baseline > gpurun_out/r3ai/no_c4.json 2> gpurun_out/r3ai/no_c4.err &&
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r3ai/full.json 2> gpurun_out/r3ai/full.err
