#!/bin/bash
# A/B of the GEMM engine: census + bench with the in-tree library vs $1 (default _exp/head)
#   PYTEST_K="gemm" bash tools/gemm_ab.sh _exp/head   (runs those gpu tests first)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ALT=${1:-_exp/head}
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$PYTEST_K" > gpurun_out/ab_tests.txt 2>&1 || { tail -30 gpurun_out/ab_tests.txt; exit 1; }
  tail -2 gpurun_out/ab_tests.txt
fi
timeout -k 10 300 python tools/gemm_census.py --top 25 > gpurun_out/census_cur.txt 2>&1
ACCUNET_LIB_OVERRIDE=$PWD/$ALT/libaccunet_hip.so timeout -k 10 300 python tools/gemm_census.py --top 25 > gpurun_out/census_alt.txt 2>&1
for d in ${DTYPES:-fp32}; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dtype $d > gpurun_out/bench_cur_$d.txt 2>&1
  ACCUNET_LIB_OVERRIDE=$PWD/$ALT/libaccunet_hip.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dtype $d > gpurun_out/bench_alt_$d.txt 2>&1
done
for f in cur alt; do echo "== $f"; head -${CENSUS_LINES:-16} gpurun_out/census_$f.txt; grep -o '"value": [0-9.]*' gpurun_out/bench_${f}_*.txt; done
