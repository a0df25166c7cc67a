#!/bin/bash
# SE A/B: GPU tests touching SE, then bench fp32 + bf16 with the fused middle step,
# unfused (ACCUNET_SE_FUSED=0) and the library in $1 (default _exp/head)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ALT=${1:-_exp/head}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-se or model}" > gpurun_out/se_tests.txt 2>&1 || { tail -40 gpurun_out/se_tests.txt; exit 1; }
tail -2 gpurun_out/se_tests.txt
for d in ${DTYPES:-fp32}; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dtype $d > gpurun_out/se_cur_$d.txt 2>&1
  ACCUNET_SE_FUSED=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dtype $d > gpurun_out/se_unf_$d.txt 2>&1
  ACCUNET_LIB_OVERRIDE=$PWD/$ALT/libaccunet_hip.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dtype $d > gpurun_out/se_alt_$d.txt 2>&1
done
for f in gpurun_out/se_cur_* gpurun_out/se_unf_* gpurun_out/se_alt_*; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"K3[^}]*' $f | head -c 300)"; done
