#!/bin/bash
# 128x64 tiles for K <= 64, N > 96 (ACCUNET_K64_TILE_B): GEMM / model tests, then whole-step A/B fp32 + bf16
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 240 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -n 1 gpurun_out/gputests.log
for rep in 1 2; do
  for dt in fp32 bf16; do
    for v in 1 0; do
      ACCUNET_K64_TILE_B=$v timeout -k 10 400 python bench.py --dtype $dt --no-cpu-baseline --no-probe > gpurun_out/bench_k64_${dt}_$v.log 2>&1
      echo "$dt k64tileB=$v rep $rep: $(grep -o '"value": [0-9.]*' gpurun_out/bench_k64_${dt}_$v.log)"
    done
  done
done
