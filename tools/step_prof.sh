#!/bin/bash
# rocprofv3 kernel trace of short fp32 and bf16 bench runs -> per-step kernel table
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in ${DTYPES:-fp32 bf16}; do
  rm -rf gpurun_out/sp_$d
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sp_$d -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-probe --dtype $d > gpurun_out/sp_$d.log 2>&1
  python tools/step_profile.py gpurun_out/sp_$d --top ${TOP:-45} > gpurun_out/step_$d.txt
  rm -rf gpurun_out/sp_$d
  head -3 gpurun_out/step_$d.txt
done
