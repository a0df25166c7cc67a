#!/bin/bash
# Same-box A/B: current tree vs the library in $1 (default _ab/head, tools/build_alt.sh),
# bench.py --dtype $DT (default bf16) with the roofline probes, alternating, twice each.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ALT=${1:-_ab/head}
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 240 --timeout-method thread -k "$PYTEST_K" > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
  tail -1 gpurun_out/ab_tests.log
fi
for dt in ${DTS:-bf16}; do
  for i in 1 2; do
    for v in cur alt; do
      if [ $v = alt ]; then export ACCUNET_LIB_OVERRIDE=$PWD/$ALT/libaccunet_hip.so; else unset ACCUNET_LIB_OVERRIDE; fi
      timeout -k 10 300 python bench.py --no-cpu-baseline --dtype $dt > gpurun_out/ab_$v$i.log 2>&1
      echo "$dt $v$i $(grep '^{"metric' gpurun_out/ab_$v$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], [(r['kernel'][:16], r['avg_us']) for r in d['rooflines']])")"
    done
  done
done
