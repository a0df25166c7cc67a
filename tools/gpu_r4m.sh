#!/bin/bash
# halo forward: stagger A/B (ACCUNET_C3_STAGGER = s_sleep(32) count for the grid's second half)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/c3_stagger.txt
for rep in 1 2; do
  for v in 0 2 4 8; do
    echo "== ACCUNET_C3_STAGGER=$v" >> gpurun_out/c3_stagger.txt
    ACCUNET_C3_STAGGER=$v GB_ONLY="rspth1 3x3 fwd" timeout -k 10 120 tools/gbench 40 >> gpurun_out/c3_stagger.txt 2>&1
  done
done
cat gpurun_out/c3_stagger.txt
