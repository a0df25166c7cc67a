#!/bin/bash
set -e -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
tail -n 3 gpurun_out/gputests.log
timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2>&1 || { tail -30 gpurun_out/bench_full.log; exit 1; }
grep '^{"metric' gpurun_out/bench_full.log | cut -c1-400
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/bench_full.log") if l.startswith('{"metric')][0])
print("value", d["value"], "roofline", json.dumps(d["roofline"])[:600])
for r in d.get("rooflines", []):
    print(json.dumps({k: r.get(k) for k in ("kernel", "avg_us", "median_us", "frac", "timing")})[:400])
print("dw_se", d.get("roofline_dw_se"))
PY
