"""Split-K reduce census from a rocprofv3 kernel trace (round-5 verdict item 6): every
splitk_reduce dispatch attributed to the kernel that ran right before it on the same
stream (its GEMM: exact in a single-stream trace, ACCUNET_WGRAD_STREAM=0), grouped by
(GEMM kernel, GEMM grid, reduce grid); per group: launches, total and mean duration.
Dual-stream traces stretch a reduce that waits for CU slots behind the other stream's
persistent kernels, so compare families on single-stream traces.

    python tools/splitk_census.py gpurun_out/pa_ss [--steps 7]
"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--steps", type=int, default=7, help="steps in the trace (per-step totals)")
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    prev, agg = {}, collections.defaultdict(list)
    for r in rows:
        n = r["Kernel_Name"].replace("void ", "")
        g = f'{r["Grid_Size_X"]}x{r["Grid_Size_Y"]}x{r["Grid_Size_Z"]}'
        if "splitk_reduce" in n:
            p = prev.get(r["Stream_Id"], ("?", ""))
            agg[(p[0].split("(")[0][:48], p[1], r["Grid_Size_X"])].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        else:
            prev[r["Stream_Id"]] = (n, g)
    tot = sum(sum(v) for v in agg.values())
    nl = sum(len(v) for v in agg.values())
    print(f"split-K reduces: {nl} launches, {tot / 1e3:.3f} ms in the trace, "
          f"{tot / 1e3 / a.steps:.3f} ms and {nl / a.steps:.0f} launches per step ({a.steps} steps)")
    print(f"{'ms/step':>8s} {'n/step':>6s} {'us':>7s}  reduce grid  after GEMM (grid)")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{sum(v) / 1e3 / a.steps:8.3f} {len(v) / a.steps:6.1f} {sum(v) / len(v):7.1f}  "
              f"{k[2]:>11s}  {k[0]} ({k[1]})")


if __name__ == "__main__":
    main()
