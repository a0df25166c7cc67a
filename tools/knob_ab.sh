#!/bin/bash
# Census + bench under values of one environment knob: KNOB=NAME VALUES="a b c"
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in $VALUES; do
  env $KNOB=$v timeout -k 10 300 python tools/gemm_census.py --top 200 > gpurun_out/census_k$v.txt 2>&1
  env $KNOB=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe > gpurun_out/bench_k$v.txt 2>&1
  echo "== $KNOB=$v"; head -2 gpurun_out/census_k$v.txt | tail -1; grep -o '"value": [0-9.]*' gpurun_out/bench_k$v.txt
done
