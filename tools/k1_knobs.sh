#!/bin/bash
# K1 tuning-knob sweep (csrc/dwconv.hip getenv knobs) with tools/kbench
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 5 120 tools/kbench 40 > gpurun_out/kn_$name.txt 2>&1
  printf "%-14s %s | %s | %s\n" "$name" "$(grep 'K1 dw3x3_fwd 16x' gpurun_out/kn_$name.txt | awk '{print $5}')" \
    "$(grep 'K1 bf16' gpurun_out/kn_$name.txt | awk '{print $6}')" "$(grep 'flat' gpurun_out/kn_$name.txt | awk '{print $5}')"
}
echo "name           fp32_us | bf16_us | flatcopy_us"
run base X=1
run cg0 ACCUNET_DW_CGFAST=0
run rch2 ACCUNET_DW_RCH_FORCE=2
run rch4 ACCUNET_DW_RCH_FORCE=4
run rch8 ACCUNET_DW_RCH_FORCE=8
run rch32 ACCUNET_DW_RCH_FORCE=32
run ntl0 ACCUNET_DW_NTL=0
run noremap ACCUNET_DW_NOREMAP=1
run base2 X=1
