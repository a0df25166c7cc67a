"""ISA audit of the HIP kernels: for every kernel of csrc/*.hip, the s_waitcnt
vmcnt(0) count inside loops (a full drain of outstanding loads AND stores, the
usual sign that a conditional load/store or a pending prologue load defeated the
compiler's counting: each one is an HBM/L2 round trip per iteration), stores
inside loops, VGPRs, scratch and occupancy.

    python tools/isa_audit.py [--filter dw3x3] [--dir /tmp/isa]
"""
import argparse
import glob
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "acc-unet-unext_amd", "csrc")


def compile_all(out, only):
    os.makedirs(out, exist_ok=True)
    procs = []
    for src in sorted(glob.glob(os.path.join(CSRC, "*.hip"))):
        base = os.path.basename(src)
        if only and not any(o in base for o in only):
            continue
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--offload-device-only",
               "-S", "-I", os.path.join(ROOT, "include"), "-I", CSRC, src,
               "-o", os.path.join(out, base + ".s")]
        procs.append(subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL))
        if len(procs) >= 8:
            procs.pop(0).wait()
    for p in procs:
        p.wait()


def audit(path, filt):
    s = open(path).read()
    rows = []
    for m in re.finditer(r"^(_Z\w+):", s, re.M):
        name = m.group(1)
        if filt and filt not in name:
            continue
        end = s.find(".Lfunc_end", m.end())
        body = s[m.end():end].split("\n")
        meta = s[end:s.find(".end_amdhsa_kernel", end) if ".end_amdhsa_kernel" in s[end:] else end + 4000]
        loop, vm0, vmn, st = False, 0, 0, 0
        for l in body:
            if "Loop Header" in l:
                loop = True
            if not loop:
                continue
            if re.search(r"s_waitcnt vmcnt\(0\)", l):
                vm0 += 1
            elif re.search(r"s_waitcnt vmcnt\(\d+\)", l):
                vmn += 1
            if re.search(r"(global|buffer)_store", l):
                st += 1
        rows.append((name, vm0, vmn, st, loop))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--filter", default="")
    ap.add_argument("--only", nargs="*", default=[])
    ap.add_argument("--dir", default="/tmp/isa")
    a = ap.parse_args()
    compile_all(a.dir, a.only)
    print(f"{'vmcnt0':>6} {'vmcntN':>6} {'stores':>6}  kernel (counts after the first loop header)")
    for f in sorted(glob.glob(os.path.join(a.dir, "*.s"))):
        if a.only and not any(o in os.path.basename(f) for o in a.only):
            continue
        for name, vm0, vmn, st, loop in audit(f, a.filter):
            if not loop:
                continue
            dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
            print(f"{vm0:6d} {vmn:6d} {st:6d}  {os.path.basename(f)[:-6]}: {dem[:110]}")


if __name__ == "__main__":
    sys.exit(main())
