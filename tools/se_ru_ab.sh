#!/bin/bash
# A/B of the SE forward reduce's rows in flight per thread (ACCUNET_SE_RU 8 / 16):
# kbench's K3 line and the fp32 step, alternating; the SE GPU tests under 16
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 env ACCUNET_SE_RU=16 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -k "se_layer" --timeout 120 --timeout-method thread > gpurun_out/se_ru_tests.log 2>&1 || { tail -30 gpurun_out/se_ru_tests.log; exit 1; }
tail -n 1 gpurun_out/se_ru_tests.log
for i in 1 2 3; do
  for ru in 8 16; do
    echo "RU=$ru $(ACCUNET_SE_RU=$ru timeout -k 10 120 tools/kbench 20 | grep 'K3 se_fwd')"
  done
done
for i in 1 2; do
  for ru in 8 16; do
    ACCUNET_SE_RU=$ru timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > gpurun_out/se_ru_$ru.log 2>&1
    echo "RU=$ru step $(grep -o '"value": [0-9.]*' gpurun_out/se_ru_$ru.log | head -1)"
  done
done
