"""Per-kernel summary (calls, total/avg ms, share) from a rocprofv3 kernel-trace,
either run_kernel_stats.csv/run_kernel_trace.csv or a rocpd sqlite run_results.db.

    python tools/kstats.py gpurun_out/prof2 [--top 40] [--steps N]
"""
import argparse
import collections
import csv
import glob
import os
import sqlite3


def load(d):
    db = glob.glob(os.path.join(d, "**", "*results.db"), recursive=True)
    rows = collections.defaultdict(list)
    if db:
        c = sqlite3.connect(db[0])
        for name, dur in c.execute("select name, duration from kernels"):
            rows[name].append(dur)
        return rows
    tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    with open(tr[0]) as f:
        for r in csv.DictReader(f):
            rows[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--steps", type=int, default=0, help="divide totals by this many steps")
    a = ap.parse_args()
    rows = load(a.dir)
    tot = sum(sum(v) for v in rows.values())
    div = a.steps if a.steps else 1
    print(f"total kernel time {tot / 1e6 / div:.2f} ms" + (" per step" if a.steps else ""))
    print(f"{'ms':>9} {'calls':>7} {'avg_us':>9} {'%':>6}  kernel")
    for name, v in sorted(rows.items(), key=lambda kv: -sum(kv[1]))[:a.top]:
        s = sum(v)
        print(f"{s / 1e6 / div:9.3f} {len(v) // div:7d} {s / len(v) / 1e3:9.1f} {100 * s / tot:6.2f}  {name[:110]}")


if __name__ == "__main__":
    main()
