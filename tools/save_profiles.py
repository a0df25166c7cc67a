"""Copy the judged summaries of one GPU round (tools/gpu_round.sh, results merged
into gpurun_out/) into profiles/, named per round:

    python tools/save_profiles.py r01

  {r}_bench_kernel_stats.csv  rocprofv3 --stats of bench.py --steps 5 --warmup 2
  {r}_bench_kstats.txt        per-kernel totals of that trace (tools/kstats.py)
  {r}_step_breakdown.txt      one graph-replayed step of that trace: time by kernel
                              family, launches, inter-kernel gaps
  {r}_k1_trace.txt            K1 (cnv12 dw3x3, 16x256x256x96) dispatches: the 20-launch
                              roofline probe (must agree with bench.py's roofline.avg_us)
                              and the in-model launches
  {r}_pmc_k1.csv              FETCH_SIZE / WRITE_SIZE rows of the probe's K1 dispatches
  k1_traffic.json             tools/pmc_traffic.py on those passes (bench.py reads it)
  {r}_kbench.txt              tools/kbench (kernels + float4 copy ceilings)
  {r}_bench_line.json         the bench.py JSON line of the round
"""
import collections
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")
K1 = "dw3x3_tile_fwd_kernel<8, false>"

FAMILIES = ["gemm_f32", "splitk", "dw3x3", "dw_wgrad", "bn_bwd", "bn_fin", "affine_act",
            "se_", "hanc_pyramid", "pool", "colreduce", "sum_rows", "CUDAFunctor_add",
            "copyBuffer", "group_relayout", "permute", "blocksum", "adam", "loss", "head",
            "slice_copy", "pixel_shuffle"]


def family(name):
    if "elementwise_kernel" in name and "add" in name:
        return "autograd add (gradient accumulation)"
    for k in FAMILIES:
        if k in name:
            return k
    return name.split("(")[0][:40]


def trace_rows():
    f = glob.glob(os.path.join(OUT, "prof_bench", "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def dur(r):
    return int(r["End_Timestamp"]) - int(r["Start_Timestamp"])


def step_breakdown(rows):
    idx = [i for i, r in enumerate(rows) if "adam" in r["Kernel_Name"]]
    s, e = idx[-2] + 1, idx[-1] + 1  # the last full step (replay + Adam) before the probes
    seg = rows[s:e]
    cat, cnt = collections.Counter(), collections.Counter()
    for r in seg:
        k = family(r["Kernel_Name"])
        cat[k] += dur(r)
        cnt[k] += 1
    busy = sum(cat.values())
    wall = int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])
    lines = [f"one training step (HIP-graph replay + Adam) from the rocprofv3 kernel trace",
             f"kernels {len(seg)}, wall {wall / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms, "
             f"gaps {(wall - busy) / 1e6:.2f} ms", "", "     ms      %  launches  family"]
    for k, v in cat.most_common():
        lines.append(f"{v / 1e6:7.2f} {100 * v / busy:6.1f} {cnt[k]:9d}  {k}")
    return "\n".join(lines) + "\n"


def k1_trace(rows):
    k = [r for r in rows if K1 in r["Kernel_Name"] and r["Grid_Size_X"] == "65536"
         and r["Grid_Size_Y"] == "3"]
    probe = k[-20:]
    pavg = sum(dur(r) for r in probe) / len(probe)
    # cnv21's depthwise (16x128x128x96) launches the same 256x3 grid in ~1/4 the time
    inm = [r for r in k[:-20] if dur(r) > 0.5 * pavg]
    other = [r for r in k[:-20] if dur(r) <= 0.5 * pavg]
    avg = lambda rs: sum(dur(r) for r in rs) / max(len(rs), 1) / 1e3
    lines = ["rocprofv3 --kernel-trace of `python bench.py --steps 5 --warmup 2 --no-cpu-baseline`",
             f"{K1}, grid 256x3 workgroups (16x256x256x96: cnv12 / cnv92 forward)",
             f"  last 20 dispatches = bench.py roofline probe: avg {avg(probe):.2f} us "
             f"({805306368 / (avg(probe) * 1e-6) / 1e9:.0f} GB/s)",
             f"  in-model dispatches of the same shape (cnv12 / cnv92 forward inside the "
             f"graph-replayed steps): {len(inm)}, avg {avg(inm):.2f} us",
             f"  same grid, other shape (cnv21 depthwise, 16x128x128x96): {len(other)}, "
             f"avg {avg(other):.2f} us", "", "  dispatch durations (us):"]
    lab = lambda r: "probe" if r in probe else ("in-model cnv12/92" if r in inm else "cnv21")
    lines += [f"    {dur(r) / 1e3:8.2f}  {lab(r)}" for r in k]
    return "\n".join(lines) + "\n"


def main():
    r = sys.argv[1]
    os.makedirs(PROF, exist_ok=True)
    st = glob.glob(os.path.join(OUT, "prof_bench", "**", "*kernel_stats.csv"), recursive=True)[0]
    shutil.copy(st, os.path.join(PROF, f"{r}_bench_kernel_stats.csv"))
    ks = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "kstats.py"),
                         os.path.join(OUT, "prof_bench"), "--top", "60"],
                        capture_output=True, text=True, check=True).stdout
    open(os.path.join(PROF, f"{r}_bench_kstats.txt"), "w").write(ks)
    rows = trace_rows()
    open(os.path.join(PROF, f"{r}_step_breakdown.txt"), "w").write(step_breakdown(rows))
    open(os.path.join(PROF, f"{r}_k1_trace.txt"), "w").write(k1_trace(rows))
    # PMC rows of the probe's K1 dispatches + the traffic summary bench.py reads
    out = []
    for d in ("pmc_fetch", "pmc_write"):
        f = glob.glob(os.path.join(OUT, d, "**", "*counter_collection.csv"), recursive=True)[0]
        rs = [x for x in csv.DictReader(open(f)) if K1 in x["Kernel_Name"]
              and x["Grid_Size"] == "196608"]
        rs.sort(key=lambda x: int(x["Dispatch_Id"]))
        out += rs[-20:]
    with open(os.path.join(PROF, f"{r}_pmc_k1.csv"), "w", newline="") as fo:
        w = csv.DictWriter(fo, fieldnames=list(out[0].keys()))
        w.writeheader()
        w.writerows(out)
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"),
                    os.path.join(OUT, "pmc_fetch"), os.path.join(OUT, "pmc_write"), K1, "196608",
                    "20", os.path.join(PROF, "k1_traffic.json"), "16x256x256x96"],
                   check=True, capture_output=True)
    if os.path.exists(os.path.join(OUT, "kbench.txt")):
        shutil.copy(os.path.join(OUT, "kbench.txt"), os.path.join(PROF, f"{r}_kbench.txt"))
    for line in open(os.path.join(OUT, "bench_full.log")):
        if line.startswith('{"metric"'):
            open(os.path.join(PROF, f"{r}_bench_line.json"), "w").write(line)
    print("saved", r)


if __name__ == "__main__":
    main()
