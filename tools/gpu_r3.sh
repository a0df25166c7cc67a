#!/bin/bash
# Round-3 GPU pass: K1 access-shape lab, kbench, the -m gpu suite, then a same-box
# bench A/B of the tree against _ab/head (tools/build_alt.sh) when it exists.
# Each GPU step has its own time limit; the first failure ends the pass.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -x tools/k1lab ] && [ -z "${SKIP_LAB:-}" ]; then
  timeout -k 10 120 tools/k1lab 20 > gpurun_out/k1lab.txt 2>&1; cat gpurun_out/k1lab.txt
fi
if [ -x tools/kbench ] && [ -z "${SKIP_KB:-}" ]; then
  timeout -k 10 120 tools/kbench 20 > gpurun_out/kbench.txt 2>&1; cat gpurun_out/kbench.txt
fi
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 800 python -u -m pytest tests -q -m gpu -x --timeout 240 --timeout-method thread -k "${PYTEST_K:-}" > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
  tail -2 gpurun_out/gputests.log
fi
if [ -f _ab/head/libaccunet_hip.so ] && [ -z "${SKIP_AB:-}" ]; then
  DTS="${DTS:-fp32}" bash tools/ab_lib.sh _ab/head
fi
