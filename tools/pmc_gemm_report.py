"""Summarise tools/pmc_gemm.sh: per replayed GEMM (the last REPS GEMM dispatches of
each run) the MFMA pipe utilisation, wave-state split, effective clock and HBM
traffic.

  MFMA util   = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
                (GRBM_GUI_ACTIVE is summed over the 8 XCDs; 256 CUs x 4 SIMDs)
  clock       = GRBM_GUI_ACTIVE / 8 / dispatch duration
  traffic     = FETCH_SIZE x 2 (gfx950 counts 128-B wide reads at 64 B:
                /opt/skills/guides/MI355X_MICROARCH.md, HBM section) + WRITE_SIZE, KiB -> B

    python tools/pmc_gemm_report.py gpurun_out/pmc_gemm [--reps 20]
"""
import argparse
import collections
import csv
import glob
import os
import re
import statistics

# the GEMM engines and the ResPath 3x3 direct convolutions (csrc/conv3x3.hip) that a
# replayed GEMM key may dispatch to
GEMM_PREFIXES = ("void gemm_", "gemm_", "void conv3x3_", "conv3x3_")


def load(path, reps):
    """{dispatch_id: {counter: value, 'name', 'dur_ns', 'grid'}} of the last reps GEMM dispatches"""
    rows = collections.OrderedDict()
    with open(path) as f:
        for r in csv.DictReader(f):
            d = rows.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"],
                                                         "dur_ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                                         "grid": int(r["Grid_Size"])})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    g = [v for k, v in rows.items() if v["name"].startswith(GEMM_PREFIXES)]
    return g[-reps:]


def shrink(path, reps):
    """rewrite a counter CSV keeping only the rows of its last reps GEMM dispatches"""
    with open(path) as f:
        rd = csv.DictReader(f)
        fields = rd.fieldnames
        rows = list(rd)
    ids = []
    for r in rows:
        d = int(r["Dispatch_Id"])
        if r["Kernel_Name"].startswith(GEMM_PREFIXES) and (not ids or ids[-1] != d):
            ids.append(d)
    keep = set(ids[-reps:])
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=fields)
        w.writeheader()
        for r in rows:
            if int(r["Dispatch_Id"]) in keep:
                w.writerow(r)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--shrink", action="store_true")
    a = ap.parse_args()
    if a.shrink:
        return shrink(a.dir, a.reps)
    print(f"{'#':>2} {'us':>8} {'TF/s':>6} {'MFMAutil':>8} {'clkGHz':>6} {'wait%':>6} {'issue%':>6} "
          f"{'fetchMB':>8} {'writeMB':>8}  shape / kernel")
    for i in range(64):
        sq = os.path.join(a.dir, f"g{i}_sq", "run_counter_collection.csv")
        if not os.path.exists(sq):
            break
        log = open(os.path.join(a.dir, f"g{i}_sq.log")).read()
        m = re.search(r"replayed #\d+ (\(.*?\)) x\d+: ([0-9.e+]+) flop", log)
        shape, flop = (m.group(1), float(m.group(2))) if m else ("?", 0.0)
        s = load(sq, a.reps)
        dur = statistics.median(d["dur_ns"] for d in s) * 1e-9
        gui = statistics.median(d.get("GRBM_GUI_ACTIVE", 0) for d in s)
        busy = statistics.median(d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) for d in s)
        wc = statistics.median(d.get("SQ_WAVE_CYCLES", 0) for d in s) or 1
        wait = statistics.median(d.get("SQ_WAIT_ANY", 0) for d in s) / wc
        winst = statistics.median(d.get("SQ_WAIT_INST_ANY", 0) for d in s) / wc
        cyc = gui / 8
        util = busy / (cyc * 1024) if cyc else 0
        clk = cyc / dur / 1e9 if dur else 0
        fetch = write = float("nan")
        fp = os.path.join(a.dir, f"g{i}_fetch", "run_counter_collection.csv")
        wp = os.path.join(a.dir, f"g{i}_write", "run_counter_collection.csv")
        if os.path.exists(fp):
            fetch = statistics.median(d.get("FETCH_SIZE", 0) for d in load(fp, a.reps)) * 1024 * 2 / 1e6
        if os.path.exists(wp):
            write = statistics.median(d.get("WRITE_SIZE", 0) for d in load(wp, a.reps)) * 1024 / 1e6
        print(f"{i:2d} {dur * 1e6:8.1f} {flop / dur / 1e12 if dur else 0:6.1f} {util:8.3f} {clk:6.2f} "
              f"{100 * wait:6.1f} {100 * winst:6.1f} {fetch:8.1f} {write:8.1f}  {shape} {s[-1]['name'][:60]}")


if __name__ == "__main__":
    main()
