"""Per-step kernel profile from a rocprofv3 kernel trace of bench.py: takes the
windows between consecutive launches of a marker kernel (one per training step,
default the loss forward) over the last --last steps, so setup / capture / probe
kernels are excluded.

    python tools/step_profile.py gpurun_out/prof_bench [--last 4] [--top 40]
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
    ap.add_argument("--last", type=int, default=4)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    tr = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    ev = []
    with open(tr) as f:
        for r in csv.DictReader(f):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ev.sort()
    marks = [i for i, e in enumerate(ev) if e[2].startswith(a.marker)]
    marks = marks[-(a.last + 1):]
    n = len(marks) - 1
    rows = collections.defaultdict(list)
    busy = 0
    union = 0  # time with any kernel running (two streams: durations overlap)
    for s, e in zip(marks[:-1], marks[1:]):
        cs = ce = None
        for t0, t1, k in ev[s:e]:
            rows[k].append(t1 - t0)
            busy += t1 - t0
            if ce is None or t0 > ce:
                if ce is not None:
                    union += ce - cs
                cs, ce = t0, t1
            else:
                ce = max(ce, t1)
        if ce is not None:
            union += ce - cs
    wall = (ev[marks[-1]][0] - ev[marks[0]][0]) / n
    print(f"{n} steps: wall {wall / 1e6:.2f} ms/step, GPU busy {union / n / 1e6:.2f} ms/step, "
          f"kernel time sum {busy / n / 1e6:.2f} ms/step, "
          f"launches {sum(len(v) for v in rows.values()) / n:.0f}/step")
    out = sorted(((sum(v) / n, len(v) / n, sum(v) / len(v), k) for k, v in rows.items()), reverse=True)
    for t, c, avg, k in out[:a.top]:
        print(f"{t / 1e3:9.1f} us {c:6.1f} x {avg / 1e3:7.1f} us  {k[:100]}")


if __name__ == "__main__":
    main()
