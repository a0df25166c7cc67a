"""Live per-kernel timing with HIP events (used by bench.py for the roofline line).

Events are recorded on torch's current HIP stream — the stream every accunet
kernel is launched on — around selected launches, only while enabled. Each tag
groups launches of one kernel at one shape; `rooflines()` turns the average
launch duration into achieved algorithmic GB/s (or TFLOP/s) against a peak.
"""
from __future__ import annotations

from collections import defaultdict
from contextlib import contextmanager

import torch

_enabled = False
_events = defaultdict(list)   # tag -> [(start, end)]
_meta = {}                    # tag -> dict(bytes=, flops=, kernel=, shape=)


def enable(on: bool = True):
    global _enabled
    _enabled = on
    if on:
        _events.clear()


def enabled() -> bool:
    return _enabled


@contextmanager
def region(tag: str, *, kernel: str, shape: str, bytes_alg: float = 0.0, flops: float = 0.0):
    if not _enabled:
        yield
        return
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    try:
        yield
    finally:
        e.record()
        _events[tag].append((s, e))
        _meta[tag] = dict(kernel=kernel, shape=shape, bytes=bytes_alg, flops=flops)


def summary():
    torch.cuda.synchronize()
    out = []
    for tag, evs in _events.items():
        ms = [s.elapsed_time(e) for s, e in evs]
        avg = sum(ms) / len(ms)
        m = _meta[tag]
        out.append(dict(tag=tag, launches=len(ms), avg_us=1000.0 * avg, total_ms=sum(ms), **m))
    out.sort(key=lambda r: -r["total_ms"])
    return out


def rooflines(hbm_peak_gbs: float, mfma_peak_tflops: float = 157.3):
    rows = []
    for r in summary():
        t = r["avg_us"] * 1e-6
        if r["bytes"] > 0:
            ach = r["bytes"] / t / 1e9
            rows.append({"bound": "hbm", "achieved": round(ach, 1), "peak": hbm_peak_gbs,
                         "unit": "GB/s", "frac": round(ach / hbm_peak_gbs, 4), "traffic": None,
                         "kernel": r["kernel"], "shape": r["shape"], "avg_us": round(r["avg_us"], 2),
                         "launches": r["launches"], "bytes_alg_per_launch": r["bytes"],
                         "share_of_tracked_ms": round(r["total_ms"], 3)})
        elif r["flops"] > 0:
            ach = r["flops"] / t / 1e12
            rows.append({"bound": "mfma", "achieved": round(ach, 2), "peak": mfma_peak_tflops,
                         "unit": "TFLOP/s", "frac": round(ach / mfma_peak_tflops, 4),
                         "traffic": None, "kernel": r["kernel"], "shape": r["shape"],
                         "avg_us": round(r["avg_us"], 2), "launches": r["launches"],
                         "flops_alg_per_launch": r["flops"],
                         "share_of_tracked_ms": round(r["total_ms"], 3)})
    return rows
