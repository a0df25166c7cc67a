"""Kernel sequence of one training step from a rocprofv3 kernel trace: every dispatch
between two consecutive launches of the marker kernel (default the loss forward), in
start order, with its offset from the step start, duration, queue / stream and grid,
plus per-name counts -- to see where a variant's extra dispatches sit in the step.

    python tools/step_seq.py gpurun_out/pa_b16dp [--step -2] [--grep copyBuffer]
"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--marker", default="loss_reduce_kernel")
    ap.add_argument("--step", type=int, default=-2, help="which marker window (python index)")
    ap.add_argument("--grep", default="", help="only list dispatches whose name contains this")
    ap.add_argument("--context", type=int, default=0, help="also list N dispatches around a match")
    a = ap.parse_args()
    tr = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    with open(tr) as f:
        ev = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(ev) if r["Kernel_Name"].startswith(a.marker)]
    s, e = marks[a.step - 1], marks[a.step]
    t0 = int(ev[s]["Start_Timestamp"])
    win = ev[s:e]
    hit = [i for i, r in enumerate(win) if a.grep in r["Kernel_Name"]] if a.grep else range(len(win))
    show = sorted({j for i in hit for j in range(i - a.context, i + a.context + 1) if 0 <= j < len(win)})
    for i in show:
        r = win[i]
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{i:5d} {(st - t0) / 1e3:10.1f} us {(en - st) / 1e3:8.1f} us q{r.get('Queue_Id', '?'):>3} "
              f"s{r.get('Stream_Id', '?'):>3} grid {r.get('Grid_Size_X', r.get('Grid_Size', '?'))} "
              f"{r['Kernel_Name'][:100]}")
    cnt = collections.Counter(r["Kernel_Name"][:60] for r in win)
    print(f"# {len(win)} dispatches, step {(int(ev[e]['Start_Timestamp']) - t0) / 1e3:.1f} us")
    for k, n in cnt.most_common(12):
        print(f"# {n:5d} {k}")


if __name__ == "__main__":
    main()
