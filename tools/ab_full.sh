#!/bin/bash
# Whole GPU suite, then bench fp32 + bf16 of the tree vs the library in $1 (default _exp/head)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ALT=${1:-_exp/head}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/ab_tests.txt 2>&1 || { tail -40 gpurun_out/ab_tests.txt; exit 1; }
tail -1 gpurun_out/ab_tests.txt
for d in ${DTYPES:-fp32 bf16}; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe --dtype $d > gpurun_out/ab_cur_$d.txt 2>&1
  ACCUNET_LIB_OVERRIDE=$PWD/$ALT/libaccunet_hip.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe --dtype $d > gpurun_out/ab_alt_$d.txt 2>&1
done
for f in gpurun_out/ab_cur_* gpurun_out/ab_alt_*; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
