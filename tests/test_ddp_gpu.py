"""The data-parallel gradient exchange with GPU gradients: two ranks on cuda:0
(a one-GPU box cannot host two RCCL ranks, so the process group is gloo,
which all-reduces CUDA tensors through the host), running the real
GradAllReduce -- gradients as views of persistent flat buckets, buckets
launched in index order from post-accumulate-grad hooks, the 1/world scale a
libmdemi sweep per bucket -- around a tiny NeW-CRFs train step.  The mean of the per-rank gradients must equal the
per-shard gradients averaged on one replica, and every rank must end with the
same gradients.  RCCL itself only differs in the transport."""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
H, W = 64, 96


def _rendezvous():
    """A fresh file:// rendezvous (no TCP port to race for)."""
    fd, path = tempfile.mkstemp(prefix="mdemi_gloo_gpu_")
    os.close(fd)
    os.unlink(path)
    return path


def _model_and_shard(rank):
    from mdemi.model.NewCRFs import NewCRFDepth
    from oracle.weights import closed_form_fill, rng_array
    m = NewCRFDepth(version="tiny07", max_depth=10.0, drop_path_rate=0.0)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    closed_form_fill(sd, seed=0.9, scale=0.02)
    m.load_state_dict(sd)
    img = torch.from_numpy(rng_array((1, 3, H, W), 40 + rank)).float()
    g = torch.Generator().manual_seed(80 + rank)
    gt = torch.rand(1, 1, H, W, generator=g) * 9.0 + 0.5
    return m, img, gt


def _worker(rank, world, path, q):
    import sys
    for p in (ROOT, os.path.join(ROOT, "monocular-depth-estimation_amd")):
        sys.path.insert(0, p)
    try:
        dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from mdemi.train import GradAllReduce, SILogLoss, broadcast_parameters
        m, img, gt = _model_and_shard(rank)
        m = m.cuda().train()
        broadcast_parameters(m)
        ar = GradAllReduce(m, bucket_mb=2.0)
        loss = SILogLoss(10.0, 0.15)(m(img.cuda()), gt.cuda())
        loss.backward()
        ar.finish()
        torch.cuda.synchronize()
        # numpy, pickled by value: torch CPU tensors would travel as shared-memory fds that die with the rank
        q.put((rank, {"grads": [p.grad.detach().cpu().numpy() for p in m.parameters()], "nbuckets": len(ar.buckets),
                      "order": ar.last_launch_order}))
        dist.destroy_process_group()
    except Exception as e:  # surface worker failures in the parent
        q.put((rank, repr(e)))


def test_grad_allreduce_gpu_gradients_two_ranks():
    from mdemi.train import SILogLoss
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    path = _rendezvous()
    procs = [ctx.Process(target=_worker, args=(r, world, path, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = dict(q.get(timeout=180) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r, v in out.items():
        assert not isinstance(v, str), f"rank {r} failed: {v}"
    assert out[0]["nbuckets"] > 2
    assert out[0]["order"] == list(range(out[0]["nbuckets"])) == out[1]["order"]
    for r in out:
        out[r]["grads"] = [torch.from_numpy(g) for g in out[r]["grads"]]
    for a, b in zip(out[0]["grads"], out[1]["grads"]):
        assert torch.equal(a, b)  # one all-reduced buffer, one scale: identical on every rank
    # single replica: per-shard gradients, averaged
    acc = None
    for r in range(world):
        m, img, gt = _model_and_shard(r)
        m = m.cuda().train()
        SILogLoss(10.0, 0.15)(m(img.cuda()), gt.cuda()).backward()
        g = [p.grad.detach().cpu().double() for p in m.parameters()]
        acc = g if acc is None else [x + y for x, y in zip(acc, g)]
    for i, (want, got) in enumerate(zip(acc, out[0]["grads"])):
        want = want / world
        err = (got.double() - want).abs().max().item()
        scale = want.abs().max().item()
        assert err <= 1e-4 * scale + 1e-9, (i, err, scale)


@pytest.mark.parametrize("capturable", [False, True])
def test_world_scale_folded_into_adamw_is_exact(capturable):
    """Trainer folds the data-parallel mean's 1/world into the AdamW step (FusedAdamW.grad_scale,
    GradAllReduce.scale_in_finish = False) instead of sweeping the reduced gradients: taking
    the gradient sums at grad_scale = 1/world -- in the clip norm and in the update -- must give
    the parameters and moments that scaling the sums first (the libmdemi sweep finish() runs)
    gives, bit for bit, over three clipped steps."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "monocular-depth-estimation_amd"))
    from mdemi import _lib as L
    from mdemi.train import FusedAdamW
    world = 4
    g = torch.Generator().manual_seed(7)
    shapes = [(300, 17), (64,), (1000,), (3, 5, 7)]
    p0 = [torch.randn(s, generator=g).cuda() for s in shapes]
    sums = [[torch.randn(s, generator=g).cuda() * 3.0 for s in shapes] for _ in range(3)]
    pa = [torch.nn.Parameter(t.clone()) for t in p0]
    pb = [torch.nn.Parameter(t.clone()) for t in p0]
    oa = FusedAdamW(pa, lr=1e-2, weight_decay=0.1, max_grad_norm=0.5, capturable=capturable)
    ob = FusedAdamW(pb, lr=1e-2, weight_decay=0.1, max_grad_norm=0.5, capturable=capturable)
    ob.grad_scale = 1.0 / world
    for step in sums:
        for p, s in zip(pa, step):
            p.grad = torch.empty_like(s)
            L.call("mdemi_elementwise", L.EW_AXPBY, s.data_ptr(), s.data_ptr(), p.grad.data_ptr(), s.numel(),
                   1.0 / world, 0.0, L.stream())
        for p, s in zip(pb, step):
            p.grad = s.clone()
        oa.step()
        ob.step()
    torch.cuda.synchronize()
    for a, b in zip(pa, pb):
        assert torch.equal(a, b)
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(oa.state[a][k], ob.state[b][k])
