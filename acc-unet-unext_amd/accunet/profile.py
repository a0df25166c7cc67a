"""Live per-kernel timing with HIP events (used by bench.py for the roofline line).

Eager mode: events are recorded on torch's current HIP stream — the stream every
accunet kernel is launched on — around selected launches, only while enabled. Each
tag groups launches of one kernel at one shape; `rooflines()` turns the average
launch duration into achieved algorithmic GB/s (or TFLOP/s) against a peak.

HIP-graph mode (the training step bench.py times): `graph_time(tag, n)` asks for the
first n launches of a tag in the next capture. While the stream captures, `region`
leaves a marker kernel before and after each of them; `graph_attach` (TrainStep,
before instantiating) replaces every marker by an event-record node with the
marker's dependencies and dependents, so no extra launch stays in the graph; while a
window is open (`graph_window`), `graph_before_replay` points those nodes at a fresh
event pair for each replay, so every launch of the timed region is measured on the
stream it runs on; `graph_rows` averages them.
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


# ---- in-graph timing ---------------------------------------------------------
_GT_TOP = 31          # marker ids taken from the top (GraphBuckets counts up from 0)
_GT_MAX_PAIRS = 4
_gt_want = {}         # tag -> launches still to mark in the next capture
_gt_meta = {}         # tag -> dict(kernel=, shape=, bytes=, flops=)
_gt_reserved = 0      # marker ids [0, reserved) belong to the gradient buckets
_gt_marks = []        # (tag, id_start, id_end) placed during the capture
_gt_nodes = []        # (tag, node_start, node_end) once attached
_gt_first = []        # the event pairs the nodes were created with
_gt_window = None     # [(tag, ev_start, ev_end)] recorded by the replays of the window
_gt_error = None


def graph_time(tag: str, launches: int = 1):
    """time the first `launches` launches of `tag` in the next graph capture"""
    _gt_want[tag] = launches


def graph_timing_requested() -> bool:
    return any(v > 0 for v in _gt_want.values())


def graph_reserve_markers(n: int):
    """marker ids below n are the caller's (TrainStep's gradient buckets)"""
    global _gt_reserved
    _gt_reserved = n


def _marking(tag: str) -> bool:
    if _gt_want.get(tag, 0) <= 0 or len(_gt_marks) >= _GT_MAX_PAIRS:
        return False
    if _GT_TOP - 2 * len(_gt_marks) - 1 < _gt_reserved:
        return False
    try:
        return torch.cuda.is_current_stream_capturing()
    except RuntimeError:
        return False


@contextmanager
def region(tag: str, *, kernel: str, shape: str, bytes_alg: float = 0.0, flops: float = 0.0):
    if _marking(tag):
        from . import kern
        k = len(_gt_marks)
        sid, eid = _GT_TOP - 2 * k, _GT_TOP - 2 * k - 1
        _gt_want[tag] -= 1
        kern.GraphEvent.mark(sid)
        yield
        kern.GraphEvent.mark(eid)
        _gt_marks.append((tag, sid, eid))
        _gt_meta[tag] = dict(kernel=kernel, shape=shape, bytes=bytes_alg, flops=flops)
        return
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


def _timed_event():
    import ctypes
    from . import kern
    h = ctypes.c_void_p()
    kern.call("accunet_event_create_timed", ctypes.byref(h))
    return h


def graph_marks_pending() -> bool:
    return bool(_gt_marks)


def graph_attach(raw_graph: int) -> int:
    """replace the marker pairs of this capture by event-record nodes (before the graph
    is instantiated); returns the number of timed launches. A failure leaves the graph
    valid (markers kept) and timing off (graph_error())."""
    import ctypes
    from . import _lib
    global _gt_error
    lib = _lib.load()
    _gt_nodes.clear()
    _gt_first.clear()
    for tag, sid, eid in _gt_marks:
        es, ee = _timed_event(), _timed_event()
        nodes = (ctypes.c_void_p * 2)()
        rc = lib.accunet_graph_time_markers(ctypes.c_void_p(raw_graph), sid, eid, es, ee, nodes)
        if rc != 0:
            _gt_error = f"accunet_graph_time_markers({sid}, {eid}) returned {rc}"
            _gt_nodes.clear()
            break
        _gt_nodes.append((tag, ctypes.c_void_p(nodes[0]), ctypes.c_void_p(nodes[1])))
        _gt_first.append((es, ee))
    _gt_marks.clear()
    _gt_want.clear()
    return len(_gt_nodes)


def graph_error():
    return _gt_error


def graph_window(on: bool):
    """open (collect one event pair per timed launch and replay) / close the window.
    Closing points the timing nodes back at the pairs they were created with, so later
    replays never record into an event graph_rows() destroys."""
    global _gt_window
    if on:
        _gt_window = []
    elif _gt_window is not None:
        _gt_closed.append(_gt_window)
        _gt_window = None
        _restore_first()


_gt_closed = []
_gt_graph = None      # the torch CUDAGraph whose nodes the window re-pointed


def _restore_first():
    global _gt_error
    if _gt_graph is None or not _gt_nodes:
        return
    import ctypes
    from . import _lib
    lib = _lib.load()
    ex = ctypes.c_void_p(_gt_graph.raw_cuda_graph_exec())
    for (tag, ns, ne), (es, ee) in zip(_gt_nodes, _gt_first):
        if (lib.accunet_graph_exec_event_set(ex, ns, es) != 0 or
                lib.accunet_graph_exec_event_set(ex, ne, ee) != 0):
            # the nodes may still name a window event: keep every window's events alive
            _gt_error = "accunet_graph_exec_event_set failed restoring the timing nodes"
            _gt_nodes.clear()
            return


_gt_keep = []         # event pairs that must outlive the process's replays


def graph_before_replay(graph) -> None:
    """point the timing nodes of `graph` (torch CUDAGraph) at fresh events for its next
    replay while a window is open"""
    global _gt_error, _gt_graph
    if _gt_window is None or not _gt_nodes:
        return
    import ctypes
    from . import _lib
    lib = _lib.load()
    _gt_graph = graph
    ex = ctypes.c_void_p(graph.raw_cuda_graph_exec())
    for tag, ns, ne in _gt_nodes:
        es, ee = _timed_event(), _timed_event()
        if (lib.accunet_graph_exec_event_set(ex, ns, es) != 0 or
                lib.accunet_graph_exec_event_set(ex, ne, ee) != 0):
            _gt_error = "accunet_graph_exec_event_set failed"
            _gt_nodes.clear()  # no more re-pointing; nodes may name any event made so far,
            _gt_keep.append((es, ee))  # so none of them is ever destroyed
            return
        _gt_window.append((tag, es, ee))


def graph_rows(hbm_peak_gbs: float):
    """per tag: the launches timed in the last closed window -> roofline rows"""
    import ctypes
    import statistics
    from . import _lib
    if not _gt_closed:
        return []
    torch.cuda.synchronize()
    lib = _lib.load()
    per = defaultdict(list)
    for tag, es, ee in _gt_closed[-1]:
        ms = ctypes.c_float()
        if lib.accunet_event_elapsed_ms(es, ee, ctypes.byref(ms)) == 0:
            per[tag].append(1000.0 * ms.value)
    rows = []
    for tag, us in per.items():
        m = _gt_meta[tag]
        avg = sum(us) / len(us)
        ach = m["bytes"] / (avg * 1e-6) / 1e9
        med = statistics.median(us)
        rows.append({"bound": "hbm", "achieved": round(ach, 1), "peak": hbm_peak_gbs,
                     "unit": "GB/s", "frac": round(ach / hbm_peak_gbs, 4), "traffic": None,
                     "kernel": m["kernel"], "shape": m["shape"], "avg_us": round(avg, 2),
                     "median_us": round(med, 2),
                     "frac_median": round(m["bytes"] / (med * 1e-6) / 1e9 / hbm_peak_gbs, 4),
                     "launch_us": [round(v, 1) for v in us], "launches": len(us),
                     "bytes_alg_per_launch": m["bytes"], "tag": tag})
    # the nodes point at their first pair again (graph_window(False)): the window's
    # events are done with once their records completed (synchronised above); after a
    # failed re-point (graph_error) the nodes may still name one of them: keep them all
    for lst in (_gt_closed if _gt_error is None else []):
        for _, es, ee in lst:
            lib.accunet_event_destroy(es)
            lib.accunet_event_destroy(ee)
    _gt_closed.clear()
    return rows
