#!/bin/bash
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 1 0; do
  ACCUNET_GEMM_G=$v timeout -k 10 400 python tools/fw_diag.py --variant ${VARIANT:-script} > gpurun_out/fw_diag_g$v.txt 2>&1
  echo "== G=$v"; cat gpurun_out/fw_diag_g$v.txt | grep -v Warning
done
