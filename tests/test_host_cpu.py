"""CPU-only checks of the host side: the C-ABI library loads and exports every
symbol include/accunet.h declares, the drop-in module tree matches the
reference's state_dict / seeded init, the LR schedule, the loud-failure policy
(no CPU fallback), and the data-parallel gradient reducer on gloo."""
import ctypes
import hashlib
import json
import os
import re
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLD = os.path.join(HERE, "golden")

from accunet import _lib, kern  # noqa: E402
from accunet.model import VARIANTS  # noqa: E402


def header_symbols():
    h = open(os.path.join(ROOT, "include", "accunet.h")).read()
    return sorted(set(re.findall(r"\b(?:int|size_t|long long)\s+(accunet_\w+)\s*\(", h)))


def test_library_loads_and_exports_every_header_symbol():
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 30
    for s in syms:
        assert hasattr(lib, s), s
    # the ctypes binding covers exactly the header
    assert sorted(_lib.declared_symbols()) == syms


def test_library_is_gfx950_code_object():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


@pytest.mark.parametrize("variant", list(VARIANTS))
def test_state_dict_matches_reference(variant):
    ref = json.load(open(os.path.join(GOLD, f"keys_{variant}.json")))
    torch.manual_seed(0)
    m = VARIANTS[variant](3, 1)
    keys = [[k, list(t.shape)] for k, t in m.state_dict().items()]
    assert keys == ref["keys"]
    assert sum(p.numel() for p in m.parameters()) == ref["n_params"]
    # same module construction order + same torch init calls => same seeded weights
    h = hashlib.sha256()
    for k, t in m.state_dict().items():
        h.update(t.detach().contiguous().numpy().tobytes())
    if ref.get("torch") == torch.__version__:
        assert h.hexdigest() == ref["init_sha256_seed0"]


def test_nets_shim_is_script_variant():
    sys.path.insert(0, os.path.join(ROOT, "acc-unet-unext_amd"))
    from nets.ACC_UNet import ACC_UNet
    m = ACC_UNet(n_channels=1, n_classes=1)
    assert m.cnv72.conv1.weight.shape[0] == 4 * 32 * 3  # inv_fctr 3 (Experiments/nets)
    assert m.last_activation is None


def test_lr_schedule_matches_reference():
    from accunet.optim import CosineAnnealingWarmRestarts, FusedAdam
    g = np.load(os.path.join(GOLD, "lr_schedule.npz"))
    p = torch.nn.Parameter(torch.zeros(1))
    opt = FusedAdam([p], lr=1e-3)
    sch = CosineAnnealingWarmRestarts(opt, T_0=10, eta_min=1e-5)
    lrs = []
    for _ in range(25):
        lrs.append(opt.param_groups[0]["lr"])
        sch.step()
    np.testing.assert_allclose(lrs, g["lrs"], rtol=1e-12)


def test_adam_step_counter_host_logic(monkeypatch):
    # host side only: the launch is stubbed, the step counter bookkeeping is real
    from accunet import optim
    calls = []
    monkeypatch.setattr(optim.kern, "adam_step", lambda *a: calls.append(a[-1]))
    ps = [torch.nn.Parameter(torch.zeros(3)) for _ in range(4)]
    for p in ps:
        p.grad = torch.zeros(3)
    opt = optim.FusedAdam(ps, lr=1e-3)
    monkeypatch.setattr(opt, "_table", lambda gi, params: (None, None, None, 0))
    for _ in range(3):
        opt.step()
    assert calls == [1, 2, 3]
    assert all(float(opt.state[p]["step"]) == 3.0 for p in ps)
    # a checkpoint round trip (separate step tensors after load) keeps counting
    sd = opt.state_dict()
    opt2 = optim.FusedAdam(ps, lr=1e-3)
    opt2.load_state_dict(sd)
    for p in ps:
        opt2.state[p]["step"] = torch.tensor(float(opt2.state[p]["step"]))
    monkeypatch.setattr(opt2, "_table", lambda gi, params: (None, None, None, 0))
    opt2.step()
    assert calls[-1] == 4 and float(opt2.state[ps[0]]["step"]) == 4.0
    # a parameter without a gradient this step keeps its count (torch.optim.Adam's
    # per-parameter step), the others advance
    ps[3].grad = None
    opt2.step()
    assert float(opt2.state[ps[0]]["step"]) == 5.0
    assert float(opt2.state[ps[3]]["step"]) == 4.0
    ps[3].grad = torch.zeros(3)
    with pytest.raises(RuntimeError):  # it now lags the group: refused, not silently mixed
        opt2.step()
    opt2.state[ps[3]]["step"] = torch.tensor(5.0)
    opt2.step()
    assert all(float(opt2.state[p]["step"]) == 6.0 for p in ps)
    # mismatched counters are refused, as before
    opt2.state[ps[1]]["step"] = torch.tensor(9.0)
    with pytest.raises(RuntimeError):
        opt2.step()


def test_host_tensors_fail_loudly():
    # no CPU fallback: a host tensor reaching a kernel wrapper raises
    a = torch.zeros(4, 4)
    with pytest.raises(_lib.AccError):
        kern.gemm(4, 4, 4, a=[a], lda=[4], b=a, ldb=4, c=a, ldc=4)


def test_forward_rejects_bad_spatial_size():
    m = VARIANTS["canonical"](3, 1, n_filts=8)
    with pytest.raises(ValueError):
        m(torch.zeros(1, 3, 40, 40))
    with pytest.raises(ValueError):
        m(torch.zeros(1, 4, 32, 32))


def test_forward_rejects_images_past_the_depthwise_limit():
    """ACC_UNet.forward names the 2 GiB per-image limit of the depthwise kernels before
    any launch: canonical cnv72 (4352 hidden channels at H/4) at 1408^2 fp32 is refused,
    1344^2 passes the check, and bf16 halves the bytes (1408^2 passes)."""
    m = VARIANTS["canonical"](3, 1)
    with pytest.raises(ValueError, match="cnv72.*2 GiB"):
        m.check_input_size(1408, 1408)
    m.check_input_size(1344, 1344)
    with pytest.raises(ValueError, match="2 GiB"):
        m(torch.zeros(1, 3, 1408, 1408))
    m.set_precision("bf16")
    m.check_input_size(1408, 1408)
    with pytest.raises(ValueError, match="cnv72"):
        m.check_input_size(2048, 2048)
    # the script preset (cnv72 inv_fctr 3) first hits the limit at a level-0 block
    s = VARIANTS["script"](3, 1)
    s.check_input_size(1408, 1408)
    with pytest.raises(ValueError, match="cnv91"):
        s.check_input_size(1680, 1680)


def _reducer_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from accunet.dist import GradBucketReducer
    torch.manual_seed(0)
    net = torch.nn.ModuleDict({
        "a": torch.nn.Linear(16, 32), "b": torch.nn.Linear(32, 8),
        "unused": torch.nn.Linear(8, 8)})  # never used: must still be flushed
    red = GradBucketReducer(net, bucket_mb=0.001)  # tiny buckets -> several collectives
    last = 3
    for it in range(last + 1):
        if it % 2 == 0:
            red.zero_grad()
            if it == 0:
                red.prepare()  # optional: the state also resets after every flush
        else:
            # optimizer.zero_grad() style (set_to_none) and no prepare(): the hooks must
            # move the fresh gradients back into the flat buffer and still reduce them
            net.zero_grad(set_to_none=True)
        g = torch.Generator().manual_seed(100 * it + rank)
        x = torch.randn(4, 16, generator=g)
        y = net["b"](torch.relu(net["a"](x))).square().mean()
        y.backward()
    # (the unused layer's gradient is None after a set_to_none zero_grad, as in torch)
    got = {k: p.grad.clone() if p.grad is not None else torch.zeros_like(p)
           for k, p in net.named_parameters()}
    # expected: average over ranks of the per-rank gradients of the last iteration
    exp = {k: torch.zeros_like(p) for k, p in net.named_parameters()}
    for r in range(world):
        net.zero_grad(set_to_none=True)
        for p in net.parameters():
            p.grad = None
        g = torch.Generator().manual_seed(100 * last + r)
        x = torch.randn(4, 16, generator=g)
        y = net["b"](torch.relu(net["a"](x))).square().mean()
        gr = torch.autograd.grad(y, [net["a"].weight, net["a"].bias, net["b"].weight,
                                     net["b"].bias])
        for k, t in zip(["a.weight", "a.bias", "b.weight", "b.bias"], gr):
            exp[k] += t / world
    err = max((got[k] - exp[k]).abs().max().item() for k in exp)
    q.put((rank, err, len(red.buckets)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_grad_bucket_reducer_gloo_world2(world):
    """the bucketed hook reducer over gloo: the mean of the ranks' gradients (pre-divided
    by the world, then summed: the graph path's PreMulSum form, also at world 3 where
    x/3 and x*(1/3) differ)"""
    import random
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = random.randint(20000, 40000)
    procs = [ctx.Process(target=_reducer_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, err, nb in res:
        assert nb > 1
        assert err < 1e-6, (rank, err)


class _BceDice(torch.nn.Module):
    """Trainer-compatible criterion on CPU (loss + the _show_dice hook it logs)."""

    def forward(self, pred, mask):
        return torch.nn.functional.binary_cross_entropy_with_logits(pred, mask)

    def _show_dice(self, pred, mask):
        p = (torch.sigmoid(pred) >= 0.5).float()
        return float((2 * (p * mask).sum() + 1e-5) / (p.sum() + mask.sum() + 1e-5))


def _trainer_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from accunet.dist import GradBucketReducer
    from accunet.trainer import Trainer
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Conv2d(3, 4, 1), torch.nn.ReLU(), torch.nn.Conv2d(4, 1, 1))
    init = [p.detach().clone() for p in net.parameters()]

    def batches(r):
        g = torch.Generator().manual_seed(7 + r)
        return [({"image": torch.randn(2, 3, 8, 8, generator=g),
                  "label": (torch.rand(2, 1, 8, 8, generator=g) < 0.4).float()}, None)
                for _ in range(2)]

    red = GradBucketReducer(net, bucket_mb=0.00001)  # ~2-element buckets: several collectives
    tr = Trainer(net, criterion=_BceDice(), optimizer=torch.optim.SGD(net.parameters(), lr=0.1),
                 lr_scheduler=None, device=torch.device("cpu"), reducer=red)
    tr.train_one_epoch(batches(rank), 0, True)
    got = torch.cat([p.detach().reshape(-1) for p in net.parameters()])
    # expected: SGD on the rank-averaged gradient of each step, replayed in-process
    ref = torch.nn.Sequential(torch.nn.Conv2d(3, 4, 1), torch.nn.ReLU(), torch.nn.Conv2d(4, 1, 1))
    with torch.no_grad():
        for p, v in zip(ref.parameters(), init):
            p.copy_(v)
    data = [batches(r) for r in range(world)]
    for step in range(2):
        gs = [torch.zeros_like(p) for p in ref.parameters()]
        for r in range(world):
            b = data[r][step][0]
            loss = _BceDice()(ref(b["image"]), b["label"])
            for acc, t in zip(gs, torch.autograd.grad(loss, list(ref.parameters()))):
                acc += t / world
        with torch.no_grad():
            for p, gg in zip(ref.parameters(), gs):
                p -= 0.1 * gg
    exp = torch.cat([p.detach().reshape(-1) for p in ref.parameters()])
    q.put((rank, float((got - exp).abs().max()), len(red.buckets)))
    dist.destroy_process_group()


def test_trainer_with_bucket_reducer_gloo_world2():
    """Trainer(reducer=GradBucketReducer): the epoch loop zeroes through the reducer,
    whose hooks all-reduce (mean) each bucket during backward, so every rank applies
    the rank-averaged gradient (accunet/trainer.py, accunet/dist.py)."""
    import random
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = random.randint(20000, 40000)
    procs = [ctx.Process(target=_trainer_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, err, nb in res:
        assert nb > 1
        assert err < 1e-6, (rank, err)


def test_bench_attaches_pmc_traffic_only_for_the_same_kernel_sources(tmp_path):
    """bench.py's roofline rows take `traffic` from the committed PMC summaries only when
    shape, dtype and the kernel-source hash match the tree (accunet.probe.attach_traffic);
    the committed K1 / K3 summaries describe this tree's sources."""
    import json
    from accunet import probe
    row = {"shape": "16x65536x32", "traffic": None}
    f = tmp_path / "t.json"
    base = {"shape": "16x65536x32", "dtype": "fp32", "traffic_bytes": 404.0}
    f.write_text(json.dumps(dict(base, src_sha=probe.src_hash(probe.K3_SOURCES))))
    assert probe.attach_traffic(dict(row), str(f), "fp32", probe.K3_SOURCES)["traffic"] == 404.0
    assert probe.attach_traffic(dict(row), str(f), "bf16", probe.K3_SOURCES)["traffic"] is None
    other = probe.attach_traffic(dict(row, shape="1x2x3"), str(f), "fp32", probe.K3_SOURCES)
    assert other["traffic"] is None
    f.write_text(json.dumps(dict(base, src_sha="0" * 16)))
    stale = probe.attach_traffic(dict(row), str(f), "fp32", probe.K3_SOURCES)
    assert stale["traffic"] is None and "traffic_stale" in stale
    assert probe.attach_traffic(dict(row), str(tmp_path / "none.json"), "fp32")["traffic"] is None
    prof = os.path.join(os.path.dirname(HERE), "profiles")
    for name, src, shape in (("k1_traffic.json", probe.K1_SOURCES, "16x256x256x96"),
                             ("k3_traffic.json", probe.K3_SOURCES, "16x65536x32")):
        got = probe.attach_traffic({"shape": shape, "traffic": None}, os.path.join(prof, name),
                                   "fp32", src)
        assert got["traffic"] is not None, (name, got)


def test_graph_buckets_respect_the_marker_table():
    """Graph-mode DP cuts one marker per bucket; the library's marker table holds 32.
    A tiny bucket_mb on ACC_UNet's 918 gradients (16.77 M elements) still gives <= 32
    buckets, covering every parameter exactly once in reverse registration order, and
    a 16 MB cut gives the 4-5 buckets bench.py runs with."""
    from accunet import kern
    from accunet.model import ACC_UNet
    from accunet.train import cut_buckets
    numels = [p.numel() for p in ACC_UNet(3, 1).parameters()]
    for mb, lo, hi in ((0.001, 2, kern.MAX_GRAPH_MARKERS), (16.0, 4, 5)):
        b = cut_buckets(numels, mb)
        assert lo <= len(b) <= hi, (mb, len(b))
        flat = [i for k in b for i in k]
        assert flat == list(reversed(range(len(numels))))
    # the bucket that seals last (the step's exposed reduce) holds at most tail_mb,
    # unless its first parameter alone is larger
    b = cut_buckets(numels, 16.0)
    assert len(b) == 5 and sum(numels[i] for i in b[-1]) * 4 <= 1 << 20
    b = cut_buckets([3, 400000, 5, 7], 16.0, tail_mb=0.001)
    assert b == [[3, 2, 1], [0]]


def test_abi_host_side_contract_without_a_device():
    """C-ABI entry points that validate their arguments (or only compute host-side
    geometry) answer without touching the device: bad arguments come back as -2
    (include/accunet.h), the per-stream ticket-bank registration rejects out-of-range
    banks and the null stream (a host-side table, no device call), and the statistics
    row count of K1 follows its strip tiling."""
    lib = _lib.load()
    fake = ctypes.c_void_p(0x1234)  # only used as a table key, never dereferenced
    assert lib.accunet_stream_ticket_bank(fake, 1) == 0
    assert lib.accunet_stream_ticket_bank(fake, 0) == 0   # re-registration overwrites
    assert lib.accunet_stream_ticket_bank(fake, 2) == -2  # out of range
    assert lib.accunet_stream_ticket_bank(fake, -1) == -2
    assert lib.accunet_stream_ticket_bank(None, 1) == -2  # null stream is always bank 0
    assert lib.accunet_stream_ticket_unregister(fake) == 0  # the fake handle leaves the table
    assert lib.accunet_stream_ticket_unregister(fake) == -2  # no longer registered
    assert lib.accunet_stream_ticket_unregister(None) == -2
    # the library was built from this header (the binding refuses any other)
    assert lib.accunet_abi_hash() == _lib.header_abi_hash()
    # bz without its BatchNorm state / statistics buffer: rejected before any launch
    one = ctypes.c_void_p(16)
    assert lib.accunet_dw3x3_fwd(one, one, None, None, None, 0, 1, one, None, 1, 8, 8, 32,
                                 one, None, 0, 0, None) == -2
    assert lib.accunet_gemm(None, None, 0, None) == -2
    # images of 2 GiB or more are refused (-1) before any launch: the depthwise kernels
    # address one image with 32-bit offsets. Canonical cnv72 (4352 hidden channels at
    # H/4) at a 1408^2 input: 352^2 x 4352 fp32 = 2.02 GiB; 1344^2 (336^2) is 1.83 GiB,
    # the same tensor in bf16 1.01 GiB
    assert lib.accunet_dw3x3_fwd(one, one, None, None, None, 0, 0, one, None, 1, 352, 352,
                                 4352, None, None, 0, 0, None) == -1
    assert lib.accunet_dw3x3_wgrad(one, one, None, None, 0, one, one, 1, 352, 352, 4352, one,
                                   0, 0, None) == -1
    assert lib.accunet_dw3x3_fwd(one, one, None, None, None, 0, 0, one, None, 1, 352, 352,
                                 4352, one, None, 0, 1, None) == -2  # bf16: bz check next
    assert lib.accunet_dw3x3_fwd(one, one, None, None, None, 0, 1, one, None, 1, 336, 336,
                                 4352, one, None, 0, 0, None) == -2
    # the decoder's up + concat: channel counts in quads, a skip tensor in the forward
    assert lib.accunet_convt_cat(one, None, one, one, 1, 2, 2, 6, 4, 0, 0, None) == -1
    assert lib.accunet_convt_cat(one, None, one, one, 1, 2, 2, 8, 6, 0, 0, None) == -1
    assert lib.accunet_convt_cat(one, None, None, one, 1, 2, 2, 8, 4, 0, 0, None) == -2
    # 16x256x256x96: one-shot tiles of 8 rows x 32 pixels -> 16 * 32 * 8 = 4096 statistics
    # rows (the strip kernel, ACCUNET_DW_OS=0: 32-row strips, 1024); cnv11's 9 channels
    # the register kernel
    os_knob = os.environ.get("ACCUNET_DW_OS", "1")
    # one-shot tiles (8 rows x 32 pixels -> 16 * 32 * 8 = 4096 rows) for the fp32 forward
    # above 256 MB by default, for every tile launch with ACCUNET_DW_OS=2; else 32-row
    # strips (1024 rows)
    os_on, os_all = os_knob != "0", os_knob == "2"
    # ACCUNET_DW_OS16=1: the one-shot launches without a BN-backward operand run 16-row
    # tiles (512 threads, 16 * 16 * 8 = 2048 rows); by default 8-row tiles (4096 rows)
    os16 = os.environ.get("ACCUNET_DW_OS16", "0") != "0"
    one_shot = 4 if os16 else 3
    assert lib.accunet_dw3x3_variant(16, 256, 256, 96, 0) == (one_shot if os_on else 1)
    assert lib.accunet_dw3x3_variant(16, 256, 256, 96, 1) == (one_shot if os_all else 1)
    assert lib.accunet_dw3x3_rows(16, 256, 256, 96, 0, 0) == (
        (2048 if os16 else 4096) if os_on else 1024)
    # the BN-backward data gradient of the same shape: strips unless ACCUNET_DW_OS=2
    assert lib.accunet_dw3x3_rows(16, 256, 256, 96, 0, 1) == (4096 if os_all else 1024)
    # 16 x 128^2 x 192 fp32 (201 MB, cached): strips by default
    assert lib.accunet_dw3x3_variant(16, 128, 128, 192, 0) == (one_shot if os_all else 1)
    # cnv72's 16 x 64^2 x 4352 (1.1 GB, but 136 channel groups per tile): strips by default
    assert lib.accunet_dw3x3_variant(16, 64, 64, 4352, 0) == (one_shot if os_all else 1)
    assert lib.accunet_dw3x3_variant(16, 128, 128, 384, 0) == (one_shot if os_on else 1)
    # bf16 (dt 1) runs 64-channel tiles where C % 64 == 0: 16-pixel tiles, twice the rows
    # of the same kernel's 32-pixel fp32 tiles
    r32, r16 = (lib.accunet_dw3x3_rows(16, 128, 128, 192, d, 0) for d in (0, 1))
    assert r32 * 2 == r16
    assert lib.accunet_dw3x3_rows(16, 256, 256, 96, 1, 0) == (
        (2048 if os16 else 4096) if os_all else 1024)
    assert lib.accunet_dw3x3_variant(16, 64, 64, 4352, 1) == (one_shot if os_all else 1)
    assert lib.accunet_dw3x3_variant(16, 256, 256, 9, 0) == 0


def test_bench_launcher_argument_logic(monkeypatch):
    """bench.py --gpus N: with no launcher around it (no WORLD_SIZE) and N > 1 it builds
    one torch.distributed.run child command on 127.0.0.1 with N ranks and the same
    arguments; --gpus 1, or a run already under a launcher, starts no child."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(os.path.dirname(HERE),
                                                                             "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    argv = ["--gpus", "8", "--steps", "5", "--warmup", "2"]
    cmd = bench.launcher_cmd(argv, 8, port=29555)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8"
    assert cmd[cmd.index("--nnodes") + 1] == "1"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29555"
    assert cmd[-len(argv) - 1].endswith("bench.py") and cmd[-len(argv):] == argv
    assert bench.launcher_cmd(["--gpus", "1"], 1) is None
    monkeypatch.setenv("WORLD_SIZE", "8")
    assert bench.launcher_cmd(argv, 8) is None
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    # relay: rank 0's one JSON line passes through, other output goes to stderr, and a
    # failing launcher's status comes back non-zero
    ok = bench.relay([sys.executable, "-c", "print('log'); print('{\"metric\": \"m\"}')"])
    assert ok == 0
    assert bench.relay([sys.executable, "-c", "import sys; sys.exit(3)"]) == 3
    assert bench.relay([sys.executable, "-c", "print('no line')"]) == 1


def test_host_abi_under_address_sanitizer():
    """the host side of the C ABI built with -fsanitize=address (host pass
    only; acc-unet-unext_amd/Makefile target `asan`) and driven by tools/asan_abi,
    which calls every entry point that answers without a device: geometry and workspace
    queries over the BASELINE shapes and ragged ones, the 64-entry ticket-bank table
    (filled, overflowed, unregistered in every position), the ABI hash, and the
    argument checks that return -2 before any launch. AddressSanitizer aborts on any
    invalid host access; the driver exits 0 only if every result matches the header."""
    import subprocess
    root = os.path.dirname(HERE)
    exe = os.path.join(root, "tools", "asan_abi")
    r = subprocess.run(["make", "-C", os.path.join(root, "acc-unet-unext_amd"), "-j8", "asan"],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0 and "0 failure(s)" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
    assert "AddressSanitizer" not in r.stderr, r.stderr[-4000:]


def _emulate_relayout(it, src):
    """numpy restatement of relayout_batch_kernel's index arithmetic for one item"""
    out = np.empty(it.total, dtype=np.float32)
    i = np.arange(it.total, dtype=np.int64)
    if it.kind in (3, 4):  # flat copy (bucket packing) times scale, kind 4 rounded to bf16
        out[:] = src * np.float32(it.scale)
        if it.kind == 4:
            out[:] = torch.from_numpy(out).to(torch.bfloat16).float().numpy()
        return out
    if it.kind == 0:
        r, off = i.copy(), np.zeros_like(i)
        for a in (3, 2, 1, 0):
            ia = r % it.d[a]
            r //= it.d[a]
            if it.flip[a]:
                ia = it.d[a] - 1 - ia
            off += ia * it.s[a]
    else:
        c = i % it.C
        t = i // it.C
        jj = t % it.J
        nn = t // it.J
        order = np.array(list(it.order), dtype=np.int64)
        off = nn * it.C * it.J + c * it.J + order[jj]
    if it.kind == 2:  # the group relayout's inverse: scatter
        out[off] = src[i]
    else:
        out[:] = src[off]
    return out


def test_bucket_packing_items():
    """The graph-mode data-parallel step packs each sealed gradient bucket with one
    batched launch (ops.DeferredRelayouts.copy, kinds 3 / 4): flat copies into the
    fp32 or bf16 wire; several flushes use consecutive segments of one item table."""
    from accunet import ops
    torch.manual_seed(4)
    d = ops.DeferredRelayouts("cpu", cap=4)
    src = [torch.randn(5, 7), torch.randn(33)]
    dst = [torch.empty(35), torch.empty(33, dtype=torch.bfloat16)]
    d.copy(src[0], dst[0])
    d.copy(src[1], dst[1], scale=0.125)  # pre-divided by the world (8): SUM = mean
    assert [it.kind for it in d.items] == [3, 4]
    for it, s_, d_, sc in zip(d.items, src, dst, (1.0, 0.125)):
        assert it.inp == s_.data_ptr() and it.out == d_.data_ptr() and it.total == s_.numel()
        got = _emulate_relayout(it, s_.reshape(-1).numpy())
        want = (s_.reshape(-1) * sc).to(d_.dtype).float().numpy()
        np.testing.assert_array_equal(got, want)
    with pytest.raises(ValueError):
        d.copy(torch.randn(3, dtype=torch.float64), torch.empty(3))


def test_weight_prep_items_reproduce_the_per_op_layouts():
    """ops.WeightPrep (the graph step's one-launch weight relayout): the AccRelayout
    items it builds for a full ACC_UNet (18 HANC grouped-column, 12 MLFC merge, 10 + 10
    ResPath 3x3 / flipped, 4 ConvT copies), fed through a numpy restatement of the
    kernel's index arithmetic, give exactly the layouts the per-op relayouts make
    (torch permutes of the reference weights), with ascending block ranges."""
    from accunet import ops
    from accunet._lib import AccRelayout
    from accunet.model import ACC_UNet
    assert ctypes.sizeof(AccRelayout) == 144  # (scale fills the former tail padding)
    torch.manual_seed(0)
    m = ACC_UNet(3, 1, n_filts=8)
    prep = ops.WeightPrep(m)
    assert prep.n == 18 + 12 + 20 + 4
    blk = [it.blk0 for it in prep._items]
    assert blk[0] == 0 and all(a < b for a, b in zip(blk, blk[1:]))
    want = {}
    for mod in m.modules():
        if isinstance(mod, torch.nn.Conv2d) and mod.kernel_size == (3, 3) and mod.groups == 1:
            w = mod.weight.detach()
            Co, Ci = w.shape[:2]
            want[(w.data_ptr(), "c3")] = w.permute(0, 2, 3, 1).reshape(Co, 9 * Ci)
            want[(w.data_ptr(), "c3f")] = w.flip(2, 3).permute(1, 2, 3, 0).reshape(Ci, 9 * Co)
        elif isinstance(mod, torch.nn.ConvTranspose2d):
            w = mod.weight.detach()
            want[(w.data_ptr(), "ct")] = w.permute(0, 2, 3, 1).reshape(w.shape[0], -1)
    for name, mod in m.named_modules():
        if name.endswith(".hnc"):
            w = mod.cnv.weight.detach()
            N, K = w.shape[:2]
            J = 2 * mod.k - 1
            order = list(ops._HANC_ORDER[mod.k])
            want[(w.data_ptr(), "hanc")] = w.reshape(N, K // J, J)[:, :, order].permute(0, 2, 1).reshape(N, K)
        if ".cnv_mrg" in name and name.endswith(".conv1"):
            w = mod.weight.detach()
            f = w.shape[0]
            want[(w.data_ptr(), "grp")] = w.reshape(f, f, 2).permute(0, 2, 1).reshape(f, 2 * f)
    assert set(want) == set(prep.bufs)
    ptr2w = {p.data_ptr(): p.detach().reshape(-1).numpy() for p in m.parameters()}
    for it, (key, buf) in zip(prep._items, prep.bufs.items()):
        assert it.out == buf.data_ptr() and it.inp == key[0]
        got = _emulate_relayout(it, ptr2w[it.inp])
        np.testing.assert_array_equal(got, want[key].reshape(-1).numpy(), err_msg=str(key))


def test_deferred_weight_gradient_relayouts_items():
    """ops.DeferredRelayouts (the captured backward's one-launch inverse relayouts): the
    items the backward helpers append for a HANC grouped-column weight gradient (kind 2,
    the inverse scatter), a ResPath 3x3 and a ConvT weight gradient (kind 0 permutes),
    fed through the numpy restatement of the kernel's index arithmetic, give the torch
    layouts the per-op relayouts produce; outside active() the helpers launch per op."""
    from accunet import ops
    torch.manual_seed(3)
    d = ops.DeferredRelayouts("cpu")
    k, N, C = 3, 6, 4
    J = 2 * k - 1
    order = list(ops._HANC_ORDER[k])
    w = torch.randn(N, C * J)  # reference layout [n][c*J + j]
    fwd = w.reshape(N, C, J)[:, :, order].permute(0, 2, 1).reshape(N, J * C)  # GEMM layout
    Co, Ci = 5, 3
    w3 = torch.randn(Co, Ci, 3, 3)
    g3 = w3.permute(0, 2, 3, 1).reshape(Co, 9 * Ci)  # [co][tap][ci]
    wt = torch.randn(Ci, Co, 2, 2)
    gt = wt.permute(0, 2, 3, 1).reshape(Ci, 4 * Co)  # [ci][d][co]
    outs = [torch.empty_like(w), torch.empty_like(w3), torch.empty_like(wt)]
    with d.active():
        assert ops._DEFER is d
        ops._wgrad_group_inverse(fwd, outs[0], N, C, J, order)
        ops._wgrad_permute(g3, outs[1], (Co, Ci, 3, 3), (9 * Ci, 1, 3 * Ci, Ci))
        ops._wgrad_permute(gt, outs[2], (Ci, Co, 2, 2), (4 * Co, 1, 2 * Co, Co))
    assert ops._DEFER is None and len(d.items) == 3
    assert [it.kind for it in d.items] == [2, 0, 0]
    assert d.destinations() == [o.data_ptr() for o in outs]
    for it, src, want in zip(d.items, (fwd, g3, gt), (w, w3, wt)):
        got = _emulate_relayout(it, src.reshape(-1).numpy())
        np.testing.assert_array_equal(got, want.reshape(-1).numpy())
