#!/bin/bash
# packed kernel vs the small loop shape across record sizes (where would the packed kernel pay)
set -o pipefail
mkdir -p gpurun_out/r3t
PROBE_MIB= timeout -k 10 700 python scripts/ab.py fixed64@1024,fixed256@2048,fixed1024,fixed2048,zipf_le1024,zipf_le2048 33,42,46 > gpurun_out/r3t/ab_sizes.jsonl 2> gpurun_out/r3t/ab.err
