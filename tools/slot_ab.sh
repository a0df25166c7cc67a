#!/bin/bash
# GradSlot A/B (same library): bench fp32 with and without shared gradient buffers
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for d in ${DTYPES:-fp32}; do
  for v in 1 0 1 0; do
    ACCUNET_GRADSLOT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe --dtype $d > gpurun_out/slot_$v.txt 2>&1
    echo "$d slots=$v $(grep -o '"value": [0-9.]*' gpurun_out/slot_$v.txt)"
  done
done
timeout -k 10 300 python tools/fill_sources.py > gpurun_out/fills.txt 2>&1
head -14 gpurun_out/fills.txt
