"""Summarise tools/pmc_k1.sh: per kernel (median over its dispatches in each pass) the
wave-state split, instruction mix, LDS / TA pressure, effective clock and HBM traffic.

  wait share   = SQ_WAIT_ANY / SQ_WAVE_CYCLES   (waves parked on s_waitcnt / barrier)
  issue stall  = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
  active       = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  VALU/wave, LDS/wave, VMEM rd/wr per wave = SQ_INSTS_* / SQ_WAVES
  clock        = GRBM_GUI_ACTIVE / 8 / dispatch duration
  traffic      = FETCH_SIZE x 2 (gfx950 counts 128-B wide reads at 64 B) + WRITE_SIZE (KiB)

    python tools/pmc_k1_report.py gpurun_out/pmc_k1
"""
import collections
import csv
import glob
import os
import re
import statistics
import sys


def short(name):
    name = re.sub(r"\(.*", "", name.replace("void ", ""))
    return name[:60]


def main(d):
    per = collections.defaultdict(lambda: collections.defaultdict(list))  # kernel -> counter -> values
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "*_p*", "run_counter_collection.csv"))):
        prog = os.path.basename(os.path.dirname(f)).rsplit("_p", 1)[0]
        acc = collections.OrderedDict()
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = (prog, short(r["Kernel_Name"]), int(r["Dispatch_Id"]))
                a = acc.setdefault(k, {"dur": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
                a[r["Counter_Name"]] = a.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for (prog, kn, _), a in acc.items():
            key = f"{prog}:{kn}"
            dur[key].append(a.pop("dur"))
            for c, v in a.items():
                per[key][c].append(v)
    med = lambda xs: statistics.median(xs) if xs else float("nan")
    print(f"{'kernel':62s} {'us':>7s} {'GHz':>5s} {'wait':>5s} {'stall':>5s} {'activ':>5s} "
          f"{'VALU/w':>7s} {'LDS/w':>6s} {'bank':>5s} {'RD/w':>5s} {'WR/w':>5s} {'SALU/w':>6s} "
          f"{'TAfull':>6s} {'MB':>7s}")
    for key in sorted(per):
        c = {k: med(v) for k, v in per[key].items()}
        us = med(dur[key]) / 1e3
        wc = c.get("SQ_WAVE_CYCLES", float("nan"))
        wv = c.get("SQ_WAVES", float("nan"))
        ghz = c.get("GRBM_GUI_ACTIVE", float("nan")) / 8 / (us * 1e3)
        mb = (2 * c.get("FETCH_SIZE", float("nan")) + c.get("WRITE_SIZE", float("nan"))) * 1024 / 1e6
        ta = (c.get("SQ_VMEM_TA_ADDR_FIFO_FULL", 0) + c.get("SQ_VMEM_TA_CMD_FIFO_FULL", 0) +
              c.get("SQ_VMEM_WR_TA_DATA_FIFO_FULL", 0)) / max(c.get("SQ_BUSY_CYCLES", 1), 1)
        bank = c.get("SQ_LDS_BANK_CONFLICT", float("nan")) / max(c.get("SQ_LDS_IDX_ACTIVE", 1), 1)
        print(f"{key[:62]:62s} {us:7.1f} {ghz:5.2f} {c.get('SQ_WAIT_ANY', float('nan')) / wc:5.2f} "
              f"{c.get('SQ_WAIT_INST_ANY', float('nan')) / wc:5.2f} "
              f"{c.get('SQ_ACTIVE_INST_ANY', float('nan')) / wc:5.2f} "
              f"{c.get('SQ_INSTS_VALU', float('nan')) / wv:7.0f} {c.get('SQ_INSTS_LDS', float('nan')) / wv:6.0f} "
              f"{bank:5.2f} {c.get('SQ_INSTS_VMEM_RD', float('nan')) / wv:5.0f} "
              f"{c.get('SQ_INSTS_VMEM_WR', float('nan')) / wv:5.0f} {c.get('SQ_INSTS_SALU', float('nan')) / wv:6.0f} "
              f"{ta:6.3f} {mb:7.1f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_k1")
