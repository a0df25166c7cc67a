#!/bin/bash
# PMC passes (MFMA busy, clock, FETCH/WRITE) of the ResPath 3x3 halo kernels and the
# pyramid data gradient at the final sources
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
KEYS="32,288,1048576,1,2 1048576,32,288,2,0 64,576,262144,1,2 65536,4352,128,0,1" timeout -k 10 1000 bash tools/pmc_gemm.sh > gpurun_out/pmc_gemm.log 2>&1
cat gpurun_out/pmc_gemm/report.txt
