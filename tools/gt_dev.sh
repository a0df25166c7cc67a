#!/bin/bash
# in-graph timing check: its GPU test, the fp32 bench line, the --dp-path line (a second
# graph replayed after the timed window), the bf16 line
set -e -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_graph_timing_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/gt_test.log 2>&1 || { tail -40 gpurun_out/gt_test.log; exit 1; }
tail -n 2 gpurun_out/gt_test.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > gpurun_out/gt_bench.log 2>&1 || { tail -30 gpurun_out/gt_bench.log; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/gt_bench.log") if l.startswith('{"metric')][0])
print("value", d["value"], "graph_timing_error", d.get("graph_timing_error"))
for r in d["rooflines"]:
    print(json.dumps({k: r.get(k) for k in ("kernel", "avg_us", "median_us", "frac", "launches", "launch_us", "timing", "traffic")})[:700])
    if "probe" in r: print("   probe", json.dumps(r["probe"])[:400])
print("dw_se", d["roofline_dw_se"])
PY
timeout -k 10 400 python bench.py --no-cpu-baseline --no-parity --dp-path > gpurun_out/gt_benchdp.log 2>&1 || { tail -30 gpurun_out/gt_benchdp.log; exit 1; }
grep -o '"dp_path": {[^}]*}' gpurun_out/gt_benchdp.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity --dtype bf16 > gpurun_out/gt_bench16.log 2>&1 || { tail -30 gpurun_out/gt_bench16.log; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/gt_bench16.log") if l.startswith('{"metric')][0])
print("bf16 value", d["value"], d.get("graph_timing_error"))
for r in d["rooflines"][:2]:
    print(json.dumps({k: r.get(k) for k in ("kernel", "avg_us", "frac", "launches")}), "probe", r.get("probe", {}).get("avg_us"))
PY
