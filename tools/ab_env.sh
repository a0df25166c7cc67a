#!/bin/bash
# Same-box A/B of a runtime switch: bench.py with env "$AB_ENV" (e.g. ACCUNET_WGRAD_STREAM=0)
# vs without, alternating, twice each, per dtype in $DTS (default "fp32 bf16").
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 240 --timeout-method thread -k "$PYTEST_K" > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
  tail -1 gpurun_out/ab_tests.log
fi
for dt in ${DTS:-fp32 bf16}; do
  for i in 1 2; do
    for v in cur alt; do
      if [ $v = alt ]; then E="$AB_ENV"; else E=""; fi
      timeout -k 10 300 env $E python bench.py --no-cpu-baseline --no-probe --dtype $dt > gpurun_out/ab_$v$i.log 2>&1
      echo "$dt $v$i [$E] $(grep '^{"metric' gpurun_out/ab_$v$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
    done
  done
done
