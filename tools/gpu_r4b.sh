#!/bin/bash
# Round-4: K1 lab (streaming geometries), then the -m gpu suite and the bench line.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 tools/k1lab 20 > gpurun_out/k1lab.txt 2>&1 || { cat gpurun_out/k1lab.txt; exit 1; }
cat gpurun_out/k1lab.txt
bash tools/gpu_r4a.sh
