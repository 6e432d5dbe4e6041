#!/bin/bash
# dump crc_batch_kernel asm + instruction histogram (build container, no GPU)
cd "$(dirname "$0")/../0-db_amd"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../include -Icsrc --cuda-device-only -S \
    -o build/crc32_hip.s csrc/crc32_hip.hip 2>&1 | grep -E "error" 
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../include -Icsrc --cuda-device-only -c \
    -o /tmp/kres.o csrc/crc32_hip.hip -Rpass-analysis=kernel-resource-usage 2>&1 | grep -A12 "crc_batch" | grep -E "Name|VGPRs:|SGPRs:|Occupancy|LDS|Spill" 
for k in $(grep -oE "^_ZN[^:]*crc_batch_kernel[^:]*" build/crc32_hip.s); do
  start=$(grep -n "^$k:" build/crc32_hip.s | cut -d: -f1)
  awk -v s=$start 'NR>=s {print} NR>s && /s_endpgm/ {exit}' build/crc32_hip.s > /tmp/k_$(echo $k | md5sum | cut -c1-6).s
  echo "== $k"; grep -oE "^\s+(v_|s_|ds_|global_|buffer_|flat_)[a-z0-9_]+" /tmp/k_$(echo $k | md5sum | cut -c1-6).s | sort | uniq -c | sort -rn | head -${TOP:-14}
done
