#!/bin/bash
# Round-4 A/B pass: K1 lab, kbench K1 register strip vs LDS-DMA ring (checksums must
# agree), dw3x3 tests on the DMA kernel, pyramid data-gradient GEMMs with the 1-row /
# 3-wave epilogue (current) vs the 2-row / 2-wave one (_ab/pyr0) per forced tile,
# then the -m gpu suite and the bench line.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 tools/k1lab 20 > gpurun_out/k1lab.txt 2>&1 || { cat gpurun_out/k1lab.txt; exit 1; }
cat gpurun_out/k1lab.txt
for v in 0 3; do
  ACCUNET_DW_DMA=$v timeout -k 10 120 tools/kbench 20 > gpurun_out/kbench_dma$v.txt 2>&1 || { cat gpurun_out/kbench_dma$v.txt; exit 1; }
  echo "== ACCUNET_DW_DMA=$v"; grep "K1 dw3x3_fwd 16x\|K1 checksum\|copy float4\|flip\|K1 bf16" gpurun_out/kbench_dma$v.txt
done
ACCUNET_DW_DMA=3 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "dw3x3" > gpurun_out/dw_dma_tests.log 2>&1 || { tail -30 gpurun_out/dw_dma_tests.log; exit 1; }
tail -n 2 gpurun_out/dw_dma_tests.log
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
