#!/bin/bash
# K1 dispatch-order sweep on the GPU box: channel-group-fastest 1-D grid (ACCUNET_DW_CGFAST),
# strip length (ACCUNET_DW_RCH_FORCE) and XCD remap (ACCUNET_DW_NOREMAP), via tools/kbench.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/k1_sweep.txt
: > $out
for cg in 0 1; do
  for rch in 1 2 4 8 16; do
    for nr in 0 1; do
      envs="ACCUNET_DW_CGFAST=$cg ACCUNET_DW_RCH_FORCE=$rch"
      [ $nr = 1 ] && envs="$envs ACCUNET_DW_NOREMAP=1"
      line=$(env $envs timeout -k 5 60 tools/kbench 20 | grep -E "^K1 dw3x3_fwd 16x256x256x96|^K1 dw3x3_fwd flip")
      echo "cg=$cg rch=$rch noremap=$nr" >> $out
      echo "$line" >> $out
    done
  done
done
cat $out
