#!/bin/bash
# bf16 GEMM census with the GB_PF=1 and GB_PF=2 libraries (abx/pf1, abx/pf2), twice each
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do
  for v in pf1 pf2; do
    ACCUNET_LIB_OVERRIDE=$PWD/abx/$v/libaccunet_hip.so timeout -k 10 300 python tools/gemm_census.py --dtype bf16 --top 80 > gpurun_out/census_${v}_$r.txt 2>&1
    head -n 3 gpurun_out/census_${v}_$r.txt
  done
done
