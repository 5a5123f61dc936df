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


def test_bucket_readiness_trace(rccl):
    """the traced step (GradAllReduce.trace_events, bench.py --ddp's
    `allreduce.overlap`) records when each bucket became ready and was launched; buckets
    launch in index order, each no earlier than it was ready, the first ones well before the
    end of backward; after the first step's bucket rebuild they also become ready in index
    order; the trace is off again afterwards and leaves the step's results alone."""
    import bench
    from mdemi.train import build_from_config
    opt = _dfv8_opt(1)
    torch.manual_seed(0)
    tr = build_from_config(copy.deepcopy(opt), device=DEV, world=1, steps_per_epoch=20, precision="bf16",
                           ddp=True, ddp_bucket_mb=0.25)
    torch.manual_seed(0)
    ref = build_from_config(copy.deepcopy(opt), device=DEV, world=1, steps_per_epoch=20, precision="bf16",
                            ddp=True, ddp_bucket_mb=0.25)
    ref.model.load_state_dict(tr.model.state_dict())
    b = [_batch(5)]
    tr.step(b)
    ref.step(b)
    ov = bench.ddp_overlap(tr, b)
    ref.step(b)
    assert tr.ddp.trace_events is False and tr.ddp._trace is None
    for (k, x), y in zip(tr.model.state_dict().items(), ref.model.state_dict().values()):
        assert torch.equal(x, y), k
    rows = ov["buckets"]
    n = len(tr.ddp.buckets)
    assert [r["bucket"] for r in rows] == list(range(n)) and n >= 4
    assert sorted(ov["ready_order"]) == list(range(n))
    for r in rows:
        assert r["launch_before_end_ms"] <= r["ready_before_end_ms"] + 1e-3, r
        assert r["launch_before_end_ms"] >= 0.0, r
    assert rows[0]["ready_before_end_ms"] > rows[-1]["ready_before_end_ms"]
    assert ov["model_exposed_ms"] >= 0.0
    # the first step regrouped the buckets in gradient-arrival order: from then on they become
    # ready in index order, so each is launched in the hook that completes it -- its launch event
    # follows its ready event on the stream (a held-back bucket of the old order waited 10-60 ms;
    # with these 0.25 MB buckets a lag under 2 ms is event jitter on a busy stream)
    assert ov["ready_order_is_index_order"], ov["ready_order"]
    lag = max(r["ready_before_end_ms"] - r["launch_before_end_ms"] for r in rows)
    assert lag < 2.0, (lag, ov["held_back_buckets"])
    print(f"{n} buckets, ready order {ov['ready_order']}, held back {ov['held_back_buckets']}, "
          f"8-GPU model exposed {ov['model_exposed_ms']} ms")


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


def test_layout_change_after_capture_drops_replay_gradients(mf_lib):
    """a single-process captured step leaves its gradients in place after each
    replay.  When a load_state_dict changes the optimizer's layout (here: one parameter's
    state dropped, so its moments restart), the trainer runs one eager step before it
    re-captures -- that step must not accumulate onto the last replay's gradients.  Eager and
    captured trainers, given the same state dict, agree bit for bit over the steps after it
    (eager re-warm-up, re-capture, replay)."""
    from mdemi.train import build_from_config
    opt = _dfv8_opt(1)
    torch.manual_seed(0)
    eager = build_from_config(copy.deepcopy(opt), device=DEV, steps_per_epoch=20, precision="bf16")
    torch.manual_seed(0)
    graph = build_from_config(copy.deepcopy(opt), device=DEV, steps_per_epoch=20, precision="bf16", graph=True)
    graph.model.load_state_dict(eager.model.state_dict())
    for s in range(3):
        b = [_batch(400 + s)]
        eager.step(b)
        graph.step(b)
    assert graph._graph is not None
    v0 = graph.optimizer.layout_version
    sd = eager.optimizer.state_dict()
    dropped = sorted(sd["state"])[len(sd["state"]) // 2]
    sd = {"state": {i: {k: v.clone() for k, v in st.items()} for i, st in sd["state"].items() if i != dropped},
          "param_groups": copy.deepcopy(sd["param_groups"])}
    eager.optimizer.load_state_dict(copy.deepcopy(sd))
    graph.optimizer.load_state_dict(copy.deepcopy(sd))
    assert graph.optimizer.layout_version != v0  # the stale-graph path is the one under test
    le = [eager.step([_batch(500 + s)]).item() for s in range(3)]
    lg = [graph.step([_batch(500 + s)]).item() for s in range(3)]
    assert graph._graph is not None and graph._graph_layout == graph.optimizer.layout_version
    assert le == lg, (le, lg)
    for (k, a), b in zip(eager.model.state_dict().items(), graph.model.state_dict().values()):
        assert torch.equal(a, b), k


@pytest.fixture(scope="module")
def mf_lib():
    from mdemi import _lib
    _lib.load()


def _large07_kitti_opt():
    """json/kitti/newcrfs/newcrfs_github_eval.json's train keys (bench.py _NEWCRFS_KITTI)."""
    return {"model": {"name": "newcrfs"}, "loss": {"alpha": 10.0, "beta": 0.15, "per_image": False},
            "dataset": {"data_type": "KITTI"}, "dataloader": {"batch_size": 2},
            "optimizer": {"lr": 2e-5, "weight_decay": 0.0},
            "scheduler": {"name": "onecycle", "pct_start": 0.3, "div_factor": 25, "final_div_factor": 100},
            "train": {"epoch": 25, "num_accum": 1, "grad_norm": 0.1},
            "eval": {"max_depth_eval": 80, "min_depth_eval": 0.001, "garg_crop": True, "eigen_crop": False}}


def test_newcrfs_large07_kitti_ddp_rccl_matches_single_process(rccl):
    """BASELINE configs[3]'s data-parallel path on RCCL: NeW-CRFs large07 (270 M parameters,
    1.08 GB of fp32 gradients) at KITTI 352x1216, batch 2, through GradAllReduce with the
    default 64 MB buckets on the world-1 "nccl" group.  Three DDP train steps (forward, SILog,
    backward whose hooks launch every bucket's RCCL all-reduce as it fills, finish(), clipped
    AdamW, OneCycle) equal three single-process steps bit for bit: losses, every weight, the
    optimizer moments and step counters; the buckets launch in index order.
    Reference: utils/dist_utils.py:31-64, utils/common_utils.py:20-21,
    model/NewCRFs/NewCRFDepth.py:123-148."""
    from mdemi.train import build_from_config
    opt = _large07_kitti_opt()
    torch.manual_seed(0)
    # drop_path 0: DropPath draws its per-sample masks from the GPU generator, which the two
    # trainers would advance alternately
    single = build_from_config(copy.deepcopy(opt), device=DEV, steps_per_epoch=100, drop_path=0.0)
    torch.manual_seed(0)
    ddp = build_from_config(copy.deepcopy(opt), device=DEV, steps_per_epoch=100, ddp=True, drop_path=0.0)
    ddp.model.load_state_dict(single.model.state_dict())
    assert single.ddp is None and ddp.ddp is not None
    grad_bytes = sum(ddp.ddp.bucket_bytes)
    # 1.082 GB in buckets that close once they reach 64 MiB, WITH the parameter that crossed the
    # mark (Swin-L's stage-3 MLP weights are 37.7 MB each), so buckets hold 64-100 MiB and the
    # count is 15 here.  (Round 5 first asserted >= 16 from 1.08 GB / 64 MiB, which ignores
    # that packing; the floor was corrected to 14 after the run showed 15.)
    assert grad_bytes >= 1.08e9 and len(ddp.ddp.buckets) >= 14, (grad_bytes, len(ddp.ddp.buckets))

    def batch(seed):  # SURVEY §8d KITTI: U(1, 80) depth at a Bernoulli(0.15) LiDAR-like mask
        g = torch.Generator().manual_seed(seed)
        img = torch.randn(2, 3, 352, 1216, generator=g)
        gt = (torch.rand(2, 1, 352, 1216, generator=g) * 79.0 + 1.0) * (torch.rand(2, 1, 352, 1216, generator=g) < 0.15)
        return img.to(DEV), gt.to(DEV)

    ls, ld = [], []
    for s in range(3):
        b = [batch(600 + s)]
        ls.append(single.step(b).item())
        ld.append(ddp.step(b).item())
        assert ddp.ddp.last_launch_order == list(range(len(ddp.ddp.buckets)))
    assert ls == ld, (ls, ld)
    for (k, a), b in zip(single.model.state_dict().items(), ddp.model.state_dict().values()):
        assert torch.equal(a, b), k
    so, do = single.optimizer.state_dict(), ddp.optimizer.state_dict()
    assert so["state"].keys() == do["state"].keys()
    for i in so["state"]:
        for k in ("exp_avg", "exp_avg_sq", "step"):
            a, b = so["state"][i][k], do["state"][i][k]
            assert (torch.equal(a, b) if torch.is_tensor(a) else a == b), (i, k)
    print(f"large07 KITTI DDP on RCCL: {len(ddp.ddp.buckets)} buckets, {grad_bytes / 1e9:.3f} GB, losses {ld}")


def test_quiesce_drains_every_nccl_group(rccl):
    """the capture precondition drains each RCCL group the captured step uses, not
    only the default one (GradAllReduce(group=...))."""
    from mdemi.train.builder import quiesce_process_group
    sub = dist.new_group([0], backend="nccl")
    t = torch.ones(1 << 16, device=DEV)
    works = [dist.all_reduce(t, group=sub, async_op=True) for _ in range(4)]
    quiesce_process_group(works, groups=(sub,))
    # real work around the sub-group's all-reduce, so the captured graph is not empty and its
    # replays are checked against fresh inputs
    x = torch.ones(1 << 16, device=DEV)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y = x * 2.0
        dist.all_reduce(y, group=sub)
        z = y + 1.0
    for v in (1.0, -3.5, 7.25):
        x.fill_(v)
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(z, torch.full_like(z, 2.0 * v + 1.0)), v
    assert torch.equal(t, torch.full_like(t, 1.0))  # world 1: the eager SUMs were identities
    dist.destroy_process_group(sub)


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
