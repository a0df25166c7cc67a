import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "acc-unet-unext_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


def product_src_hash() -> str:
    """sha256 (16 hex) over the product sources: csrc/*.hip|*.h, accunet/*.py, the C header.
    The GPU box gets no .git, so this hash ties a GPU test run to a commit."""
    files = []
    for d, exts in ((os.path.join(PKG, "csrc"), (".hip", ".h")),
                    (os.path.join(PKG, "accunet"), (".py",)),
                    (os.path.join(ROOT, "include"), (".h",))):
        files += sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(exts))
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.relpath(f, ROOT).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def pytest_sessionfinish(session, exitstatus):
    """GPU runs: record which in-tree shared objects this process mapped (the HIP path
    really ran, no fallback) with the outcome and the product-source hash, in
    gpurun_out/gputests_stamp.json (tools/save_profiles.py --gputests commits it)."""
    if "torch" not in sys.modules:
        return
    try:
        import torch
        if not torch.cuda.is_available():
            return
    except Exception:
        return
    so = set()
    try:
        with open("/proc/self/maps") as fh:
            for line in fh:
                path = line.split()[-1] if len(line.split()) >= 6 else ""
                if path.endswith(".so") and path.startswith(ROOT):
                    so.add(os.path.relpath(path, ROOT))
    except OSError:
        pass
    rep = session.config.pluginmanager.get_plugin("terminalreporter")
    counts = {}
    if rep is not None:
        for k in ("passed", "failed", "error", "skipped"):
            counts[k] = len(rep.stats.get(k, []))
    try:  # diagnostics only: never let the stamp affect the session's outcome
        out = os.path.join(ROOT, "gpurun_out")
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "gputests_stamp.json"), "w") as fh:
            json.dump({"product_src_sha": product_src_hash(), "exitstatus": int(exitstatus),
                       "counts": counts, "native_so_loaded": sorted(so),
                       "device": torch.cuda.get_device_name(0)}, fh, indent=1)
    except OSError:
        pass
