"""Copy the judged summaries of one GPU round into profiles/, named per round, each
stamped with the git commit and K1's source hash (accunet.probe.src_hash):

    python tools/save_profiles.py r02          (after tools/gpu_round3.sh and
                                                 tools/pmc_gemm.sh + census, merged
                                                 into gpurun_out/)
    python tools/save_profiles.py --shrink-pmc DIR...   (on the box: keep only the
                                                 probe dispatches of PMC passes)

  {r}_bench_line.json / {r}_bench_line_bf16.json / {r}_unext_bench_line.json
                              bench.py JSON lines (fp32, bf16, --model unext)
  {r}_bench_kernel_stats.csv  rocprofv3 --stats of bench.py --steps 5 --warmup 2
  {r}_bench_kstats.txt        per-kernel totals of that trace (tools/kstats.py)
  {r}_step_breakdown.txt      one graph-replayed step: time by kernel family, launches,
                              (and {r}_step_breakdown_bf16.txt for the bf16 mode)
                              inter-kernel gaps
  {r}_k1_trace.txt            K1 dispatches: the 20-launch roofline probe (agrees with
                              the bench line's roofline.avg_us) and the in-model ones
  {r}_pmc_k1.csv / {r}_pmc_k3.csv   FETCH_SIZE / WRITE_SIZE rows of the probes
  k1_traffic.json / k3_traffic.json tools/pmc_traffic.py on those passes
  {r}_pmc_gemm.txt            tools/pmc_gemm_report.py: MFMA busy, clock, wave states,
                              FETCH / WRITE for the top-5 GEMMs
  {r}_gemm_census.txt         tools/gemm_census.py (every GEMM of one step)
  {r}_kbench.txt              tools/kbench (kernels + float4 copy ceilings)
  {r}_gputests.txt            the -m gpu suite: counts, mapped .so files, source hash
"""
import collections
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")
# the fp32 K1 kernel of 16x256x256x96: one-shot 8-row tiles
K1 = os.environ.get("K1_KERNEL", "dw3x3_os_fwd_kernel<8, 8, false, 0, float>")
K1_GRID = 12288 * 256  # 4096 tiles (8 rows x 32 pixels) x 3 channel groups, 256 threads
K3 = ["se_reduce_kernel<4, float, true>", "se_mid_sample_kernel",
      "se_apply_kernel<4, float, true,"]

FAMILIES = ["gemm_f32g", "gemm_f32", "gemm_bf16", "splitk", "dw3x3", "reduce_finish", "bn_bwd",
            "bn_fin", "affine_act", "se_", "hanc_pyramid", "pool", "colreduce", "sum_rows",
            "CUDAFunctor_add", "copyBuffer", "group_relayout", "permute", "blocksum", "adam",
            "loss", "head", "slice_copy", "pixel_shuffle", "gemm_skinny"]


def stamp():
    sha = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], cwd=ROOT, capture_output=True,
                         text=True).stdout.strip()
    dirty = subprocess.run(["git", "status", "--porcelain", "acc-unet-unext_amd", "include",
                            "bench.py"], cwd=ROOT, capture_output=True, text=True).stdout.strip()
    sys.path.insert(0, os.path.join(ROOT, "acc-unet-unext_amd"))
    from accunet.probe import src_hash
    return f"git {sha}{' (+uncommitted)' if dirty else ''}, K1 src {src_hash()}"


def family(name):
    if "elementwise_kernel" in name and "add" in name:
        return "autograd add (gradient accumulation)"
    for k in FAMILIES:
        if k in name:
            return k
    return name.split("(")[0][:40]


def trace_rows(d="prof_bench"):
    f = glob.glob(os.path.join(OUT, d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def dur(r):
    return int(r["End_Timestamp"]) - int(r["Start_Timestamp"])


def grid(r):
    return int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])


def step_breakdown(rows, st):
    idx = [i for i, r in enumerate(rows) if "adam" in r["Kernel_Name"]]
    s, e = idx[-2] + 1, idx[-1] + 1  # the last full step (replay + Adam) before the probes
    seg = rows[s:e]
    cat, cnt = collections.Counter(), collections.Counter()
    for r in seg:
        k = family(r["Kernel_Name"])
        cat[k] += dur(r)
        cnt[k] += 1
    busy = sum(cat.values())
    t0 = min(int(r["Start_Timestamp"]) for r in seg)
    t1 = max(int(r["End_Timestamp"]) for r in seg)
    wall = t1 - t0
    # time with at least one kernel running (the backward's weight gradients run on a
    # second stream, so kernel durations overlap and their sum exceeds the wall time)
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in seg)
    union, cs, ce = 0, iv[0][0], iv[0][1]
    for a, b in iv[1:]:
        if a > ce:
            union += ce - cs
            cs, ce = a, b
        else:
            ce = max(ce, b)
    union += ce - cs
    lines = [f"one training step (HIP-graph replay + Adam) from the rocprofv3 kernel trace ({st})",
             f"kernels {len(seg)}, wall {wall / 1e6:.2f} ms, GPU busy (any kernel running) "
             f"{union / 1e6:.2f} ms, idle gaps {(wall - union) / 1e6:.2f} ms; sum of kernel "
             f"durations {busy / 1e6:.2f} ms (two streams overlap: per-kernel times include "
             f"sharing the GPU with the other stream)", "", "     ms      %  launches  family"]
    for k, v in cat.most_common():
        lines.append(f"{v / 1e6:7.2f} {100 * v / busy:6.1f} {cnt[k]:9d}  {k}")
    return "\n".join(lines) + "\n"


def k1_trace(rows, st):
    """K1 dispatches of the kernel trace. The probe is the last 20 dispatches (after the
    final Adam). In-model dispatches are matched by SHAPE through their position in the
    step, not by grid: several depthwise layers launch the same kernel with the same
    3072-workgroup grid (16x128^2x96 / x192, 16x64^2x384, ...), but in every step the
    forward depthwise layers run in model order (cnv12, cnv21, ..., cnv92; cnv11's 9
    channels and the 16^2 level use other kernels, every data gradient another template),
    so cnv12 and cnv92 (16x256x256x96) are the first and the last K1 dispatch of a step."""
    adam = [i for i, r in enumerate(rows) if "adam" in r["Kernel_Name"]]
    # (the DMA kernel is fp32-only; the strip kernel's fp32 instance ends "float>")
    isk1 = lambda r: K1 in r["Kernel_Name"] and ("dma" in K1 or "float>" in r["Kernel_Name"])
    k = [r for r in rows if isk1(r) and grid(r) == K1_GRID]
    probe = [r for r in rows[adam[-1] + 1:] if isk1(r)][-20:]
    inm, other = [], []
    for a, b in zip(adam[:-1], adam[1:]):
        seq = [r for r in rows[a + 1:b + 1] if isk1(r)]
        if len(seq) >= 2:
            ends = [seq[0], seq[-1]]
            inm += [r for r in ends if grid(r) == K1_GRID]
            other += [r for r in seq[1:-1] if grid(r) == K1_GRID]
    pavg = sum(dur(r) for r in probe) / len(probe)
    avg = lambda rs: sum(dur(r) for r in rs) / max(len(rs), 1) / 1e3
    pd = sorted(dur(r) for r in probe)
    lines = [f"rocprofv3 --kernel-trace of `python bench.py --steps 5 --warmup 2 --no-cpu-baseline` ({st})",
             f"{K1} ..., {K1_GRID // 256} workgroups (16x256x256x96: cnv12 / cnv92 forward)",
             f"  last 20 dispatches = bench.py roofline probe: avg {pavg / 1e3:.2f} us, median "
             f"{pd[len(pd) // 2] / 1e3:.2f} us ({805306368 / (pavg * 1e-9) / 1e9:.0f} GB/s at the avg)",
             f"  in-model dispatches of the same shape (the first and last K1 dispatch of each "
             f"graph-replayed step = cnv12 / cnv92 forward): {len(inm)}, avg {avg(inm):.2f} us",
             f"  same kernel and grid, other shapes (cnv21 ... cnv82 forward): {len(other)}, "
             f"avg {avg(other):.2f} us", "", "  dispatch durations (us):"]
    lab = lambda r: ("probe" if r in probe else "in-model cnv12/92" if r in inm else
                     "other shape" if r in other else "warm-up / capture")
    lines += [f"    {dur(r) / 1e3:8.2f}  {lab(r)}" for r in k]
    return "\n".join(lines) + "\n"


def shrink_pmc(dirs):
    """keep the rows of the last 300 dispatches (the probes run last)"""
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                rd = csv.DictReader(fh)
                fields, rows = rd.fieldnames, list(rd)
            ids = sorted({int(r["Dispatch_Id"]) for r in rows})
            keep = set(ids[-300:])
            with open(f, "w", newline="") as fo:
                w = csv.DictWriter(fo, fieldnames=fields)
                w.writeheader()
                w.writerows(r for r in rows if int(r["Dispatch_Id"]) in keep)
        for f in glob.glob(os.path.join(d, "**", "*agent_info.csv"), recursive=True):
            os.remove(f)


def pmc_rows(kname, last=20, grid_size=None):
    out = []
    for d in ("pmc_fetch", "pmc_write"):
        f = glob.glob(os.path.join(OUT, d, "**", "*counter_collection.csv"), recursive=True)[0]
        rs = [x for x in csv.DictReader(open(f)) if kname in x["Kernel_Name"]
              and (grid_size is None or x["Grid_Size"] == str(grid_size))]
        rs.sort(key=lambda x: int(x["Dispatch_Id"]))
        out += rs[-last:]
    return out


def write_csv(path, rows):
    with open(path, "w", newline="") as fo:
        w = csv.DictWriter(fo, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)


def traffic(kname, grid_size, shape, dtype="fp32"):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"),
                        os.path.join(OUT, "pmc_fetch"), os.path.join(OUT, "pmc_write"), kname,
                        str(grid_size), "20", "/dev/stdout", shape, dtype],
                       check=True, capture_output=True, text=True)
    return json.loads(r.stdout[:r.stdout.index("}") + 1])


def main():
    if sys.argv[1] == "--shrink-pmc":
        return shrink_pmc(sys.argv[2:])
    r = sys.argv[1]
    st = stamp()
    os.makedirs(PROF, exist_ok=True)
    # bench lines
    for log, name in (("bench_full.log", f"{r}_bench_line.json"), ("bench_bf16.log", f"{r}_bench_line_bf16.json"),
                      ("bench_dp32.log", f"{r}_bench_line_dp32.json"),
                      ("bench_unext.log", f"{r}_unext_bench_line.json"),
                      ("bench_w512.log", f"{r}_bench_line_w512.json")):
        p = os.path.join(OUT, log)
        if os.path.exists(p):
            for line in open(p):
                if line.startswith('{"metric"'):
                    d = json.loads(line)
                    d["_stamp"] = st
                    open(os.path.join(PROF, name), "w").write(json.dumps(d) + "\n")
    # trace
    stf = glob.glob(os.path.join(OUT, "prof_bench", "**", "*kernel_stats.csv"), recursive=True)
    if stf:
        shutil.copy(stf[0], os.path.join(PROF, f"{r}_bench_kernel_stats.csv"))
        ks = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "kstats.py"),
                             os.path.join(OUT, "prof_bench"), "--top", "60"],
                            capture_output=True, text=True, check=True).stdout
        open(os.path.join(PROF, f"{r}_bench_kstats.txt"), "w").write(f"# {st}\n" + ks)
        rows = trace_rows()
        open(os.path.join(PROF, f"{r}_step_breakdown.txt"), "w").write(step_breakdown(rows, st))
        # the bf16 activation mode's step (BASELINE configs[2]) from its own trace
        if glob.glob(os.path.join(OUT, "prof_bench_bf16", "**", "*kernel_trace.csv"), recursive=True):
            open(os.path.join(PROF, f"{r}_step_breakdown_bf16.txt"), "w").write(
                step_breakdown(trace_rows("prof_bench_bf16"), st + ", --dtype bf16"))
        open(os.path.join(PROF, f"{r}_k1_trace.txt"), "w").write(k1_trace(rows, st))
    # PMC: K1 and K3 traffic
    if glob.glob(os.path.join(OUT, "pmc_fetch", "**", "*counter_collection.csv"), recursive=True):
        k1rows = [x for x in pmc_rows(K1, grid_size=K1_GRID)
                  if "dma" in K1 or "float>" in x["Kernel_Name"]]
        write_csv(os.path.join(PROF, f"{r}_pmc_k1.csv"), k1rows)
        t1 = traffic(K1, K1_GRID, "16x256x256x96")
        t1["source"] = f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE of bench.py --eager ({st}); {r}_pmc_k1.csv"
        json.dump(t1, open(os.path.join(PROF, "k1_traffic.json"), "w"), indent=1)
        from accunet.probe import K3_SOURCES, src_hash
        k3 = {"kernels": {}, "shape": "16x65536x32", "stamp": st, "dtype": "fp32",
              "src_sha": src_hash(K3_SOURCES),
              "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), KiB -> bytes"}
        k3rows = []
        for kn in K3:
            rs = pmc_rows(kn)
            k3rows += rs
            f = [float(x["Counter_Value"]) for x in rs if x["Counter_Name"] == "FETCH_SIZE"]
            w = [float(x["Counter_Value"]) for x in rs if x["Counter_Name"] == "WRITE_SIZE"]
            k3["kernels"][kn] = {"fetch_bytes": 2048.0 * sum(f) / max(len(f), 1),
                                 "write_bytes": 1024.0 * sum(w) / max(len(w), 1), "dispatches": [len(f), len(w)]}
        k3["traffic_bytes"] = sum(v["fetch_bytes"] + v["write_bytes"] for v in k3["kernels"].values())
        k3["bytes_alg"] = 2.0 * 4 * 16 * 65536 * 32
        write_csv(os.path.join(PROF, f"{r}_pmc_k3.csv"), k3rows)
        json.dump(k3, open(os.path.join(PROF, "k3_traffic.json"), "w"), indent=1)
    # GEMM PMC + census
    rep = os.path.join(OUT, "pmc_gemm", "report.txt")
    if os.path.exists(rep):
        open(os.path.join(PROF, f"{r}_pmc_gemm.txt"), "w").write(
            f"# tools/pmc_gemm.sh + tools/pmc_gemm_report.py ({st})\n" + open(rep).read())
    cen = os.path.join(OUT, "census_full.txt")
    if os.path.exists(cen):
        open(os.path.join(PROF, f"{r}_gemm_census.txt"), "w").write(
            f"# python tools/gemm_census.py --top 200 ({st})\n" + open(cen).read())
    # the -m gpu suite of this tree: pass counts, the in-tree .so files the test process
    # mapped (tests/conftest.py writes gputests_stamp.json) and the product-source hash,
    # checked against this checkout's sources
    gs = os.path.join(OUT, "gputests_stamp.json")
    gl = os.path.join(OUT, "gputests.log")
    if os.path.exists(gs) and os.path.exists(gl):
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from conftest import product_src_hash
        d = json.load(open(gs))
        here = product_src_hash()
        tail = [l.rstrip() for l in open(gl) if l.strip()][-1]
        txt = (f"# python -m pytest tests -m gpu on one MI355X ({st})\n"
               f"product sources (csrc, accunet, include) sha {d['product_src_sha']} on the box, "
               f"{here} in this checkout: {'MATCH' if d['product_src_sha'] == here else 'DIFFERENT'}\n"
               f"device: {d.get('device')}\nexit status: {d['exitstatus']}\ncounts: {json.dumps(d['counts'])}\n"
               f"native libraries mapped by the test process: {', '.join(d['native_so_loaded'])}\n"
               f"pytest summary: {tail}\n")
        open(os.path.join(PROF, f"{r}_gputests.txt"), "w").write(txt)
    # K1 instruction-level PMC beside the lab structures (tools/pmc_k1.sh) and the
    # single-stream trace's split-K census / depthwise per-grid table (tools/prof_ab.sh)
    rep = os.path.join(OUT, "pmc_k1", "report.txt")
    if os.path.exists(rep):
        open(os.path.join(PROF, f"{r}_pmc_k1_insts.txt"), "w").write(
            f"# tools/pmc_k1.sh + tools/pmc_k1_report.py ({st})\n" + open(rep).read())
    parts = [os.path.join(OUT, f) for f in ("splitk_ss.txt", "kgrid_ss_splitk.txt", "kgrid_ss_dw3x3.txt",
                                             "step_ss.txt")]
    if all(os.path.exists(f) for f in parts[:1]):
        open(os.path.join(PROF, f"{r}_single_stream.txt"), "w").write(
            f"# single-stream step trace (ACCUNET_WGRAD_STREAM=0, tools/prof_ab.sh; {st})\n" +
            "\n".join(open(f).read() for f in parts if os.path.exists(f)))
    kb = os.path.join(OUT, "kbench.txt")
    if os.path.exists(kb):
        open(os.path.join(PROF, f"{r}_kbench.txt"), "w").write(f"# tools/kbench 20 ({st})\n" + open(kb).read())
    # the data-parallel step at world 1 (gpu_round.sh DPTRACE=1): host vs GPU time of the
    # plain and the DP step (tools/dp_host.py), and the dispatch census of one traced step
    # of each (tools/step_seq.py tail + tools/step_profile.py head)
    dp = [f for f in ("dp_host_fp32.txt", "dp_host_bf16.txt", "step_b16plain.txt", "step_b16dp.txt",
                      "seq_b16plain.txt", "seq_b16dp.txt") if os.path.exists(os.path.join(OUT, f))]
    if dp:
        txt = f"# data-parallel step at world 1 over RCCL ({st})\n"
        for f in dp:
            lines = open(os.path.join(OUT, f)).read().splitlines()
            if f.startswith("dp_host"):
                lines = [x for x in lines if x.startswith(("plain", "dp "))]
            elif f.startswith("seq_"):
                lines = [x for x in lines if x.startswith("#")]
            else:
                lines = lines[:16]
            txt += f"\n## {f}\n" + "\n".join(lines) + "\n"
        open(os.path.join(PROF, f"{r}_dp_world1.txt"), "w").write(txt)
    print("saved", r, st)


if __name__ == "__main__":
    main()
