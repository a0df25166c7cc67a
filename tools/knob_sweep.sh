#!/bin/bash
# Runtime-knob sweep of the training step: one bench.py line per (dtype, knob setting),
# no rebuild (the ACCUNET_* tuning knobs are read once per process). Bracketed by two
# baseline runs per dtype to show the box's drift.
#   KNOBS="ACCUNET_SPLIT_TARGET=1024 ACCUNET_FEW_TILES=128" DTYPES="fp32 bf16" tools/knob_sweep.sh
# PRETEST=1 runs the -m gpu suite first (stops on a failure).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "${PRETEST:-}" ]; then
  timeout -k 10 850 python -u -m pytest tests -q -m gpu -x --timeout 240 --timeout-method thread > gpurun_out/gputests_head.log 2>&1 || { tail -30 gpurun_out/gputests_head.log; exit 1; }
  tail -n 1 gpurun_out/gputests_head.log
fi
run() {  # name dtype [VAR=value]
  local name=$1 dt=$2 kv=${3:-}
  env $kv timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --dtype "$dt" > "gpurun_out/kn_$name.log" 2>&1
  python - "gpurun_out/kn_$name.log" "$name" "$dt" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric'):
        d = json.loads(l)
        print(sys.argv[2], sys.argv[3], round(d["value"], 2), round(d["ms_per_step"], 3), flush=True)
PY
}
for dt in ${DTYPES:-fp32}; do
  run "base_$dt" "$dt"
  for kv in ${KNOBS:-}; do run "${kv}_$dt" "$dt" "$kv"; done
  run "base2_$dt" "$dt"
done
