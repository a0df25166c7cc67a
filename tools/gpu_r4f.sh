#!/bin/bash
# Round-4: pyramid data-gradient epilogue A/B (gbench: the current 1-row / 3-wave
# epilogue vs _ab/pyr0's 2-row / 2-wave one, per forced tile), then the -m gpu suite and
# the bench line (with the same-run parity leg).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/pyr_ab.txt
for rep in 1 2; do
  for lib in cur pyr0; do
    for tile in -1 0 1 2 4; do
      if [ $lib = cur ]; then LP=""; else LP="$PWD/_ab/pyr0"; fi
      echo "== lib $lib tile $tile rep $rep" >> gpurun_out/pyr_ab.txt
      LD_LIBRARY_PATH=$LP ACCUNET_GEMM_TILE=$tile GB_ONLY="pyr dgrad" timeout -k 10 120 tools/gbench 20 >> gpurun_out/pyr_ab.txt 2>&1 || { cat gpurun_out/pyr_ab.txt; exit 1; }
    done
  done
done
cat gpurun_out/pyr_ab.txt
bash tools/gpu_r4a.sh
