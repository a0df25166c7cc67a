#!/bin/bash
# K <= 64 GEMMs over >= 65536 pixels with N >= 128: default tile (64x64) vs 128x64 (tile 1)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/k64_tile_ab.txt
for rep in 1 2; do
  for t in def 1; do
    echo "== tile $t" >> gpurun_out/k64_tile_ab.txt
    if [ $t = def ]; then unset ACCUNET_GEMM_TILE; else export ACCUNET_GEMM_TILE=$t; fi
    GB_ONLY=k64 timeout -k 10 120 tools/gbench 20 >> gpurun_out/k64_tile_ab.txt 2>&1
  done
done
cat gpurun_out/k64_tile_ab.txt
