#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3r
timeout -k 10 500 bash scripts/exit_probe.sh > gpurun_out/r3r/exit_probe.txt 2>&1
