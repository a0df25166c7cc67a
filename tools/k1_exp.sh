#!/bin/bash
# K1 experiments with tools/kbench (+ the dwconv / model parity tests)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 5 120 tools/kbench 20 > gpurun_out/kb_base.txt 2>&1
cat gpurun_out/kb_base.txt
if [ -n "${K1_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$K1_TESTS" > gpurun_out/k1_tests.txt 2>&1
  tail -5 gpurun_out/k1_tests.txt
fi
