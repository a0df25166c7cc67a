"""Per (kernel, grid) totals of one kernel family from a rocprofv3 kernel trace:
launches and time per step, mean per launch. For same-box A/B of kernel variants.

    python tools/kgrid.py TRACE_DIR FAMILY_SUBSTRING [--steps 7]
"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("family")
    ap.add_argument("--steps", type=int, default=7)
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].replace("void ", "")
        if a.family not in n:
            continue
        g = f'{r["Grid_Size_X"]}x{r["Grid_Size_Y"]}'
        agg[(n.split("(")[0][:70], g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tot = sum(sum(v) for v in agg.values())
    print(f"{a.family}: {tot / 1e3 / a.steps:.3f} ms/step, {sum(len(v) for v in agg.values()) / a.steps:.0f} launches/step")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{sum(v) / 1e3 / a.steps:8.3f} ms {len(v) / a.steps:5.1f}/step {sum(v) / len(v):8.1f} us  {k[1]:>14s}  {k[0]}")


if __name__ == "__main__":
    main()
