"""HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE),
corrected as MI355X_MICROARCH.md's HBM section prescribes: both counters are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane) streaming
read, so it is doubled; WRITE_SIZE is exact for 16 B/lane stores.

    python tools/pmc_traffic.py FETCH_DIR WRITE_DIR KERNEL_SUBSTR GRID_SIZE [OUT.json]

GRID_SIZE is rocprof's Grid_Size (total work-items) that identifies the instance.
"""
import csv
import glob
import json
import os
import sys


def load(d, kname, grid):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    vals = []
    for r in csv.DictReader(open(f)):
        if kname in r["Kernel_Name"] and r["Grid_Size"] == str(grid):
            vals.append(float(r["Counter_Value"]))
    return vals


def main():
    fd, wd, kname, grid = sys.argv[1:5]
    f = load(fd, kname, grid)
    w = load(wd, kname, grid)
    if not f or not w:
        sys.exit(f"no dispatches of {kname} with Grid_Size {grid}")
    fetch = 2.0 * 1024 * sum(f) / len(f)
    write = 1024.0 * sum(w) / len(w)
    out = {"kernel": kname, "grid_size": int(grid), "dispatches": [len(f), len(w)],
           "fetch_bytes": fetch, "write_bytes": write, "traffic_bytes": fetch + write,
           "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), KiB -> bytes"}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 5:
        with open(sys.argv[5], "w") as fo:
            json.dump(out, fo, indent=1)


if __name__ == "__main__":
    main()
