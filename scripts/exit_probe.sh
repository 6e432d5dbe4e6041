#!/bin/bash
# process exit cost vs GPU resources (scripts/exit_probe): wall of 5 runs per shape
for shape in "0 0 0 1" "2300 0 0 1" "0 2300 0 1" "2300 2300 0 1" "2300 2300 1 1" "290 290 1 8" "0 0 0 8"; do
  for i in 1 2 3 4 5; do
    s=$(date +%s%N); timeout -k 5 60 ./scripts/exit_probe $shape || echo "rc=$?"; e=$(date +%s%N)
    echo "$shape run$i $(( (e - s) / 1000000 )) ms"
  done
done
