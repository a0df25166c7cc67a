#!/bin/bash
# Round-4 K1 structure A/B (kbench, same box): the register-staged strip (default), the
# one-shot block tiles (ACCUNET_DW_BLK=16 / 8), the cross-lane strip (ACCUNET_DW_XL=1);
# the dw3x3 GPU tests under each; the pyramid data-gradient epilogue A/B (gbench, the
# current library vs _ab/pyr0); then the -m gpu suite and the bench line.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/k1_ab.txt
for rep in 1 2; do
  for cfg in "base" "ACCUNET_DW_BLK=16" "ACCUNET_DW_BLK=8" "ACCUNET_DW_XL=1"; do
    if [ "$cfg" = base ]; then E=""; else E="$cfg"; fi
    env $E timeout -k 10 120 tools/kbench 20 > gpurun_out/kb_tmp.txt 2>&1 || { cat gpurun_out/kb_tmp.txt; exit 1; }
    echo "== $cfg (rep $rep)" >> gpurun_out/k1_ab.txt
    grep "K1 dw3x3_fwd 16x\|copy float4 (same bytes as K1)\|K1 bf16\|flip" gpurun_out/kb_tmp.txt >> gpurun_out/k1_ab.txt
  done
done
cat gpurun_out/k1_ab.txt
for cfg in "ACCUNET_DW_BLK=16" "ACCUNET_DW_BLK=8" "ACCUNET_DW_XL=1"; do
  env $cfg timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "dw3x3" > gpurun_out/dw_ab_tests.log 2>&1 || { echo "$cfg"; tail -30 gpurun_out/dw_ab_tests.log; exit 1; }
  echo "$cfg: $(tail -n 1 gpurun_out/dw_ab_tests.log)"
done
: > gpurun_out/pyr_ab.txt
for lib in cur pyr0; do
  for tile in -1 0 1 2 4; do
    if [ $lib = cur ]; then LP=""; else LP="$PWD/_ab/pyr0"; fi
    echo "== lib $lib tile $tile" >> gpurun_out/pyr_ab.txt
    LD_LIBRARY_PATH=$LP ACCUNET_GEMM_TILE=$tile GB_ONLY="pyr dgrad" timeout -k 10 120 tools/gbench 20 >> gpurun_out/pyr_ab.txt 2>&1 || { cat gpurun_out/pyr_ab.txt; exit 1; }
  done
done
cat gpurun_out/pyr_ab.txt
bash tools/gpu_r4a.sh
