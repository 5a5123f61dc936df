"""RCCL on hardware and the hipGraph-captured data-parallel train step (BASELINE
configs[4]: Depthformer v8, bf16, hipGraph, data parallel).

A one-GPU box hosts a world-1 process group on the real "nccl" backend (RCCL on
ROCm), so RCCL's code path -- communicator setup, async bucket all-reduces on its
own stream, the event joins back into the compute stream -- runs here exactly as
on eight GPUs; only the ring is trivial.  The data-parallel step that
mdemi.train.Trainer captures (forward, loss, backward whose post-accumulate hooks
launch the bucketed all-reduces, finish(), clip, AdamW) must replay bit-for-bit
what the eager data-parallel step computes, over five steps, with and without
gradient accumulation (train.num_accum).  Reference: the DDP wrapper of the
missing run.py (utils/common_utils.py:20-21), utils/dist_utils.py:31-64,
model/Depthformer/depthformer_v8.py:46-75."""
import copy
import os
import tempfile

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def rccl():
    from mdemi import _lib
    _lib.load()
    if dist.is_initialized():
        pytest.skip("a process group is already initialised in this process")
    fd, path = tempfile.mkstemp(prefix="mdemi_rccl_")
    os.close(fd)
    os.unlink(path)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"file://{path}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    yield dist.group.WORLD
    dist.destroy_process_group()


def _dfv8_opt(num_accum):
    return {"model": {"name": "depthformer_v8", "hidden_dim": 64, "num_heads": 4, "num_bins": 64, "num_aux": 32,
                      "img_size": [128, 160], "bn_momentum": 0.1, "attn_drop_prob": 0.0, "drop_prob": 0.0},
            "loss": {"alpha": 10.0, "beta": 0.5, "per_image": True, "chamfer_weight": 0.1},
            "dataset": {"data_type": "NYU"}, "dataloader": {"batch_size": 2},
            "optimizer": {"lr": 3.2e-4, "weight_decay": 0.1},
            "scheduler": {"name": "onecycle", "pct_start": 0.15, "div_factor": 25, "final_div_factor": 100},
            "train": {"epoch": 1, "num_accum": num_accum, "grad_norm": 0.1},
            "eval": {"max_depth_eval": 10, "min_depth_eval": 0.001}}


def _batch(seed):
    g = torch.Generator().manual_seed(seed)
    img = torch.randn(2, 3, 128, 160, generator=g)
    gt = torch.rand(2, 1, 128, 160, generator=g) * 9.5 + 0.5
    return img.to(DEV), gt.to(DEV)


def test_rccl_world1_collectives(rccl):
    """dist_utils' API on the RCCL backend (dist_utils.py:15-89: mean = sum / world)."""
    from mdemi.utils import dist_utils as du
    t = torch.arange(6, dtype=torch.float32, device=DEV)
    assert torch.equal(du.all_reduce_tensor(t.clone(), op="mean"), t)
    assert du.all_reduce_scalar(3.5, op="sum") == pytest.approx(3.5)
    g = du.all_gather_tensor(t)
    assert len(g) == 1 and torch.equal(g[0], t)
    d = du.all_reduce_dict({"abs_rel": 0.25, "rmse": 1.5}, op="mean")
    assert d["abs_rel"] == pytest.approx(0.25) and d["rmse"] == pytest.approx(1.5)


@pytest.mark.parametrize("num_accum", [1, 2])
def test_graph_captured_ddp_step_matches_eager(rccl, num_accum):
    from mdemi.train import build_from_config
    opt = _dfv8_opt(num_accum)
    torch.manual_seed(0)
    eager = build_from_config(copy.deepcopy(opt), device=DEV, world=1, steps_per_epoch=20, precision="bf16",
                              ddp=True, ddp_bucket_mb=0.25)
    torch.manual_seed(0)
    graph = build_from_config(copy.deepcopy(opt), device=DEV, world=1, steps_per_epoch=20, precision="bf16",
                              graph=True, ddp=True, ddp_bucket_mb=0.25)
    graph.model.load_state_dict(eager.model.state_dict())
    assert eager.ddp is not None and graph.ddp is not None and len(graph.ddp.buckets) >= 4
    steps = [[_batch(10 * s + i) for i in range(num_accum)] for s in range(5)]
    le, lg = [], []
    for b in steps:  # graph: calls 1-2 eager, 3 captures + replays, 4-5 replay
        le.append(eager.step(b).item())
        lg.append(graph.step(b).item())
    assert graph._graph is not None
    assert le == lg, (le, lg)
    for (k, a), b in zip(eager.model.state_dict().items(), graph.model.state_dict().values()):
        assert torch.equal(a, b), k
    # every bucket was reduced, in index order, at capture (the order every replay repeats)
    assert graph.ddp.last_launch_order == list(range(len(graph.ddp.buckets)))
    assert graph.optimizer.step_count == eager.optimizer.step_count == 5
    assert graph.optimizer.steps == eager.optimizer.steps


def test_optimizer_resume_after_capture(rccl):
    """loading optimizer state into a trainer whose step is already captured
    must not leave the graph writing into freed state (optim.py load_state_dict copies
    in place; a changed layout forces a re-capture)."""
    from mdemi.train import build_from_config
    opt = _dfv8_opt(1)
    torch.manual_seed(0)
    eager = build_from_config(copy.deepcopy(opt), device=DEV, steps_per_epoch=20, precision="bf16")
    torch.manual_seed(0)
    graph = build_from_config(copy.deepcopy(opt), device=DEV, steps_per_epoch=20, precision="bf16", graph=True)
    graph.model.load_state_dict(eager.model.state_dict())
    for s in range(3):
        b = [_batch(100 + s)]
        eager.step(b)
        graph.step(b)
    assert graph._graph is not None
    sd = eager.optimizer.state_dict()
    sd = {"state": {i: {k: (v * 0.5 if k == "exp_avg" else v.clone()) for k, v in st.items()}
                    for i, st in sd["state"].items()}, "param_groups": copy.deepcopy(sd["param_groups"])}
    eager.optimizer.load_state_dict(sd)
    graph.optimizer.load_state_dict(sd)
    le = [eager.step([_batch(200 + s)]).item() for s in range(2)]
    lg = [graph.step([_batch(200 + s)]).item() for s in range(2)]
    assert le == lg
    for (k, a), b in zip(eager.model.state_dict().items(), graph.model.state_dict().values()):
        assert torch.equal(a, b), k


def test_capture_right_after_collectives(rccl):
    """a global-mode capture begun right after eager collectives must not race the
    process group's watchdog.  quiesce_process_group waits on the Works, then on
    ProcessGroupNCCL::waitForPendingWorks (the watchdog's lists empty) -- a condition, not a
    sleep -- and the capture that follows records and replays collectives correctly."""
    from mdemi.train.builder import quiesce_process_group
    ts = [torch.full((1 << 20,), float(i), device=DEV) for i in range(8)]
    works = [dist.all_reduce(t, async_op=True) for t in ts]
    quiesce_process_group(works)
    x = torch.ones(4096, device=DEV)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y = x * 2.0
        dist.all_reduce(y)
    for v in (1.0, 3.0):
        x.fill_(v)
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(y, torch.full_like(y, 2.0 * v))
    for i, t in enumerate(ts):
        assert torch.equal(t, torch.full_like(t, float(i)))


def test_graph_captured_ddp_step_benchmark_size(rccl):
    """BASELINE configs[4]'s own workload in the captured data-parallel step: Depthformer v8
    (hidden 256, 256 bins, 256 aux tokens) at NYU 480x640, bf16, default 64 MB buckets on the
    world-1 RCCL group, batch 2: the eager and the captured step agree bit for bit over 5 steps
    (calls 1-2 eager, 3 captures, 3-5 replay) -- losses, every weight, the step counters."""
    from mdemi.train import build_from_config
    opt = _dfv8_opt(1)
    opt["model"].update(hidden_dim=256, num_bins=256, num_aux=256, img_size=[480, 640])
    torch.manual_seed(0)
    eager = build_from_config(copy.deepcopy(opt), device=DEV, world=1, steps_per_epoch=20, precision="bf16",
                              ddp=True)
    torch.manual_seed(0)
    graph = build_from_config(copy.deepcopy(opt), device=DEV, world=1, steps_per_epoch=20, precision="bf16",
                              graph=True, ddp=True)
    graph.model.load_state_dict(eager.model.state_dict())

    def batch(seed):
        g = torch.Generator().manual_seed(seed)
        return (torch.randn(2, 3, 480, 640, generator=g).to(DEV),
                (torch.rand(2, 1, 480, 640, generator=g) * 9.5 + 0.5).to(DEV))

    le, lg = [], []
    for s in range(5):
        b = [batch(300 + s)]
        le.append(eager.step(b).item())
        lg.append(graph.step(b).item())
    assert graph._graph is not None
    assert le == lg, (le, lg)
    for (k, a), b in zip(eager.model.state_dict().items(), graph.model.state_dict().values()):
        assert torch.equal(a, b), k
    assert graph.optimizer.steps == eager.optimizer.steps
