"""HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE),
corrected as MI355X_MICROARCH.md's HBM section prescribes: both counters are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane) streaming
read, so it is doubled; WRITE_SIZE is exact for 16 B/lane stores.

    python tools/pmc_traffic.py FETCH_DIR WRITE_DIR KERNEL_SUBSTR GRID_SIZE LAST [OUT.json] [SHAPE] [DTYPE]

GRID_SIZE is rocprof's Grid_Size (total work-items); LAST keeps only the last N
matching dispatches in dispatch order (bench.py's roofline probe re-launches K1 20
times after the timed steps, so LAST=20 isolates exactly the probed instance even
when other layers share the grid size).
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
            vals.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    vals.sort()
    return [v for _, v in vals]


def _src_sha():
    """K1's source hash (accunet.probe.src_hash): bench.py attaches the traffic only
    to a tree with the same sources"""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "acc-unet-unext_amd"))
    from accunet.probe import src_hash
    return src_hash()


def main():
    fd, wd, kname, grid, last = sys.argv[1:6]
    f = load(fd, kname, grid)[-int(last):]
    w = load(wd, kname, grid)[-int(last):]
    if not f or not w:
        sys.exit(f"no dispatches of {kname} with Grid_Size {grid}")
    fetch = 2.0 * 1024 * sum(f) / len(f)
    write = 1024.0 * sum(w) / len(w)
    out = {"kernel": kname, "grid_size": int(grid), "dispatches": [len(f), len(w)],
           "fetch_bytes": fetch, "write_bytes": write, "traffic_bytes": fetch + write,
           "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), KiB -> bytes",
           "shape": sys.argv[7] if len(sys.argv) > 7 else None,
           "dtype": sys.argv[8] if len(sys.argv) > 8 else "fp32",
           "src_sha": _src_sha(),
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE of bench.py --eager (profiles/)"}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 6:
        with open(sys.argv[6], "w") as fo:
            json.dump(out, fo, indent=1)


if __name__ == "__main__":
    main()
