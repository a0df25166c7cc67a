#!/bin/bash
# the driver's round-end sequence at HEAD: smoke(), then bench.py with its defaults
set -e -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -n 2 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_head.log 2>&1 || { tail -30 gpurun_out/bench_head.log; exit 1; }
grep '^{"metric' gpurun_out/bench_head.log > gpurun_out/bench_head_line.json
python - <<'PY'
import json
d = json.load(open("gpurun_out/bench_head_line.json"))
r = d["roofline"]
print("value", round(d["value"], 2), "K1", r["avg_us"], r["frac"], "traffic", r.get("traffic"), "dw_se", d["roofline_dw_se"]["frac"])
c = d["cpu_baseline"]
print("cpu", c["value"], c.get("spread"), c["sample"][:160], "parity", c.get("parity", {}).get("ok"))
PY
