#!/bin/bash
# A/B of the narrow-tile (128x32) LDS-DMA ring depth: tools/gbench over the ResPath 3x3
# and other narrow shapes with the in-tree library (3 stages) and _ab/stg{4,6,8}
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/stg_ab.txt
for rep in 1 2; do
  for v in base stg4 stg6 stg8; do
    if [ $v = base ]; then LP=""; else LP="$PWD/_ab/$v"; fi
    echo "== $v (rep $rep)" >> gpurun_out/stg_ab.txt
    for f in rspth narrow "cnv92 pyr"; do
      LD_LIBRARY_PATH=$LP GB_ONLY="$f" timeout -k 10 120 tools/gbench 20 >> gpurun_out/stg_ab.txt 2>&1
    done
  done
done
cat gpurun_out/stg_ab.txt
