#!/bin/bash
# Same-box A/B of several libraries / env settings on bench.py, round-robin $REPS times:
#   VARIANTS="name:libdir:ENV=val,ENV2=val ..."  (libdir "-" = the in-tree library;
#   other libraries from tools/build_alt.sh or tools/build_flags.sh under _ab/)
#   DT=fp32|bf16 (default fp32), BENCH_ARGS (extra bench.py arguments, e.g. --no-probe)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in ${REPS:-1 2}; do
  for v in $VARIANTS; do
    IFS=: read -r name lib envs <<< "$v"
    if [ "$lib" = "-" ]; then unset ACCUNET_LIB_OVERRIDE; else export ACCUNET_LIB_OVERRIDE=$PWD/$lib/libaccunet_hip.so; fi
    timeout -k 10 300 env ${envs//,/ } python bench.py --no-cpu-baseline --dtype ${DT:-fp32} ${BENCH_ARGS:-} > gpurun_out/ab_$name$rep.log 2>&1
    echo "$name$rep $(grep '^{"metric' gpurun_out/ab_$name$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], [(r['kernel'][:18], r['avg_us'], r['frac']) for r in d.get('rooflines', [])])")"
  done
done
