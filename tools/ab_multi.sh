#!/bin/bash
# Same-box A/B/C... of runtime switches: bench.py once per configuration in $AB_ENVS
# (';'-separated env assignments, "" = the defaults), round-robin $AB_REPS times
# (default 2), per dtype in $DTS (default fp32). Each run has its own time limit and
# the first failure ends the pass.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS=';' read -r -a CFGS <<< "${AB_ENVS:-}"
[ ${#CFGS[@]} -eq 0 ] && CFGS=("")
for dt in ${DTS:-fp32}; do
  for i in $(seq 1 "${AB_REPS:-2}"); do
    for j in "${!CFGS[@]}"; do
      E="${CFGS[$j]}"
      timeout -k 10 300 env $E python bench.py --no-cpu-baseline --no-probe --dtype $dt ${AB_ARGS:-} > gpurun_out/abm_$j.log 2>&1
      echo "$dt rep$i cfg$j [$E] $(grep '^{"metric' gpurun_out/abm_$j.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
    done
  done
done
