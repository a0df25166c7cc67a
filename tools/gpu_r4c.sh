#!/bin/bash
# Round-4 K1 A/B: lab geometries, kbench with the register-staged strip (default) and
# the LDS-DMA ring (ACCUNET_DW_DMA=1, checksums must agree), dw3x3 GPU tests on the DMA
# kernel, then the -m gpu suite and the bench line.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 tools/k1lab 20 > gpurun_out/k1lab.txt 2>&1 || { cat gpurun_out/k1lab.txt; exit 1; }
cat gpurun_out/k1lab.txt
for v in 0 1 0 1; do
  ACCUNET_DW_DMA=$v timeout -k 10 120 tools/kbench 20 > gpurun_out/kbench_dma$v.txt 2>&1 || { cat gpurun_out/kbench_dma$v.txt; exit 1; }
  echo "== ACCUNET_DW_DMA=$v"; grep "K1 dw3x3_fwd 16x\|K1 checksum\|copy float4 (same bytes as K1)\|flip" gpurun_out/kbench_dma$v.txt
done
ACCUNET_DW_DMA=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k dw3x3 > gpurun_out/dw_dma_tests.log 2>&1 || { tail -30 gpurun_out/dw_dma_tests.log; exit 1; }
tail -2 gpurun_out/dw_dma_tests.log
bash tools/gpu_r4a.sh
