"""Checkpoint interop on the GPU path: an upstream-format NeW-CRFs
checkpoint -- the `{'model': {'module.<key>': ...}}` container that
checkpoint/newcrfs_checkpoint_rename.py reads, saved from a window-12 model -- is renamed
(rename_newcrfs_checkpoint), loaded into the window-7 tiny07 model by load_checkpoint
(newcrf_utils.py:194-264: 'module.' strip, non-strict load, bicubic resize of every
relative_position_bias_table of the backbone from 23x23 to 13x13, newcrf_utils.py:245-260), and the
resulting model's forward through libmdemi matches the fp64 oracle run on the same
loaded state dict (1e-4 relative, the north_star depth bar)."""
from collections import OrderedDict

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_window12_rename_format_checkpoint_into_tiny07_forward():
    from mdemi.model.NewCRFs import NewCRFDepth
    from mdemi.utils import checkpoint as ck
    from oracle import newcrfs as onc
    from oracle.weights import closed_form_fill, rng_array

    src_model = NewCRFDepth(version="tiny12", max_depth=10.0, drop_path_rate=0.0)
    src = OrderedDict((k, v.clone()) for k, v in src_model.state_dict().items())
    closed_form_fill(src, seed=0.9, scale=0.02)
    upstream = {"model": OrderedDict(("module." + k, v) for k, v in src.items()
                                     if "relative_position_index" not in k)}
    renamed = ck.rename_newcrfs_checkpoint(upstream)
    assert all(not k.startswith("module.") for k in renamed["model"])

    m = NewCRFDepth(version="tiny07", max_depth=10.0, drop_path_rate=0.0)
    ck.load_checkpoint(m, renamed, strict=False)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    # every bias table came from the checkpoint through the bicubic resize
    n_tab = 0
    for k, v in sd.items():
        if "relative_position_bias_table" not in k:
            continue
        t = src[k]
        if t.shape[0] == 169:  # the NeW-CRF decoder's window is 7 in every version
            assert torch.equal(v, t), k
            continue
        want = F.interpolate(t.permute(1, 0).reshape(1, t.shape[1], 23, 23), size=(13, 13), mode="bicubic")
        assert torch.equal(v, want.reshape(t.shape[1], 169).permute(1, 0)), k
        n_tab += 1
    assert n_tab == 12  # the tiny backbone's 2 + 2 + 6 + 2 blocks
    # every other same-shaped tensor loaded unchanged
    for k, v in sd.items():
        if k in src and "relative_position" not in k and src[k].shape == v.shape:
            assert torch.equal(v, src[k]), k

    m = m.to(DEV).train()  # training-mode BatchNorm, as the oracle
    img = torch.from_numpy(rng_array((2, 3, 64, 96), 41))
    with torch.no_grad():
        depth = m(img.float().to(DEV)).double().cpu()
    ref = onc.newcrf_depth({k: v.double() if torch.is_floating_point(v) else v for k, v in sd.items()},
                           img.double(), "tiny07", max_depth=10.0)
    err = (depth - ref).abs().max().item()
    assert err <= 1e-4 * ref.abs().max().item(), err


@pytest.mark.parametrize("graph", [False, True])
def test_training_state_resume_is_bit_exact(tmp_path, graph):
    """save_checkpoint after 2 train steps of tiny07 (64x96, clipped AdamW, OneCycle), then 2
    more steps, equals a fresh Trainer resumed from that file (Trainer.resume: weights,
    FusedAdamW moments and per-parameter steps, OneCycle position) taking the same 2 steps --
    bit for bit, eager and hipGraph-captured (utils/common_utils.py:12-31)."""
    from mdemi.model.NewCRFs import NewCRFDepth
    from mdemi.train import FusedAdamW, OneCycleLR, SILogLoss
    from mdemi.train.builder import Trainer

    g = torch.Generator().manual_seed(3)
    data = [(torch.randn(2, 3, 64, 96, generator=g).to(DEV), (torch.rand(2, 1, 64, 96, generator=g) * 9 + 0.5).to(DEV))
            for _ in range(4)]
    loss = SILogLoss(10.0, 0.15)

    def trainer(seed):
        torch.manual_seed(seed)
        m = NewCRFDepth(version="tiny07", max_depth=10.0, drop_path_rate=0.0).to(DEV).train()
        opt = FusedAdamW(m.parameters(), lr=2e-4, weight_decay=0.01, max_grad_norm=0.1, capturable=graph)
        sched = OneCycleLR(opt, max_lr=2e-4, total_steps=10, pct_start=0.3)
        return Trainer({"train": {}}, m, loss, opt, sched, graph=graph)

    a = trainer(0)
    for i in range(2):
        a.step([data[i]])
    a.save("mid", str(tmp_path), 2, 0.0)
    for i in range(2, 4):
        a.step([data[i]])
    b = trainer(1)
    b.resume(str(tmp_path / "mid.pth"))
    for i in range(2, 4):
        b.step([data[i]])
    torch.cuda.synchronize()
    assert b.optimizer.step_count == a.optimizer.step_count == 4
    assert b.scheduler.last_step == a.scheduler.last_step
    for (k, pa), pb in zip(a.model.state_dict().items(), b.model.state_dict().values()):
        assert torch.equal(pa, pb), k
