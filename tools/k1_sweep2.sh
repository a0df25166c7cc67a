#!/bin/bash
# K1: non-temporal input loads x channel-group-fastest grid, default strip length (tools/kbench).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/k1_sweep2.txt
: > $out
for rep in 1 2; do
for cg in 0 1; do
  for ntl in 0 1; do
    line=$(ACCUNET_DW_CGFAST=$cg ACCUNET_DW_NTL=$ntl timeout -k 5 60 tools/kbench 40 | grep -E "^K1 dw3x3_fwd 16x256x256x96|^K1 dw3x3_fwd flip")
    echo "cg=$cg ntl=$ntl" >> $out
    echo "$line" >> $out
  done
done
done
cat $out
