"""CPU checks of host-side pieces added around the hot path: the oracle's
bin chamfer restatement on a hand-worked case (the loss module is absent from
the reference, so this pins the restatement to its published definition) and
the RunningAverage(Dict) mirror (utils/common_utils.py:92-135)."""
import torch

from mdemi.utils.common_utils import RunningAverage, RunningAverageDict
from oracle.adabins import bins_chamfer_loss


def test_chamfer_oracle_hand_worked():
    # edges 0,1,2,3 -> centres .5 1.5 2.5; targets .5, 2.4 (0.0 is below 1e-3: dropped)
    e = torch.tensor([[0.0, 1.0, 2.0, 3.0]], dtype=torch.float64, requires_grad=True)
    gt = torch.tensor([[[[0.5, 2.4, 0.0]]]], dtype=torch.float64)
    loss = bins_chamfer_loss(e, gt)
    # cham_x = (0 + 0.81 + 0.01) / 3 ; cham_y = (0 + 0.01) / 2
    assert abs(loss.item() - ((0.81 + 0.01) / 3 + 0.01 / 2)) < 1e-12
    loss.backward()
    # dL/dc = (2/3)(c - t*) + (2/2) sum_{t -> c}(c - t): c0: 0, c1: (2/3)(-0.9), c2: (2/3)(0.1) + (0.1)
    gc = torch.tensor([0.0, -0.6, 2 / 3 * 0.1 + 0.1], dtype=torch.float64)
    want = torch.zeros(4, dtype=torch.float64)
    want[:3] += 0.5 * gc
    want[1:] += 0.5 * gc
    assert torch.allclose(e.grad[0], want, atol=1e-12)
    # the centres form gives the same loss
    c = 0.5 * (e.detach()[:, 1:] + e.detach()[:, :-1])
    assert abs(bins_chamfer_loss(c.view(1, 3, 1, 1), gt, from_edges=False).item() - loss.item()) < 1e-12


def test_running_average_dict():
    r = RunningAverage()
    for v in (1.0, torch.tensor(2.0), 6.0):
        r.append(v)
    assert r.count == 3 and abs(r.avg - 3.0) < 1e-12
    d = RunningAverageDict()
    d.reset()  # no-op before the first update, as in the reference
    d.update({"a1": 0.5, "rmse": 2.0})
    d.update({"a1": 1.0, "rmse": 4.0})
    assert d.get_value() == {"a1": 0.75, "rmse": 3.0}
    d.reset()
    d.update({"a1": 0.25, "rmse": 1.0})
    assert d.get_value() == {"a1": 0.25, "rmse": 1.0}


def test_split_k_plan():
    """Split-K planning (mdemi.functional._split_for): no split once >= 384 output tiles fill the
    chip or the reduction is short; skinny outputs split deep; bf16 keeps >= 256 K rows per
    split where fp32 keeps >= 512 (profiles/round4/ab_split_min_rows.txt)."""
    from mdemi import functional as mf
    assert mf._split_for(9600, 3072, 768) == 1          # 75 x 24 tiles
    assert mf._split_for(128, 128, 400) == 1            # 25 K tiles: too short to split
    fp32 = mf._split_for(768, 128, 9600)                # 6 tiles, 600 K tiles
    assert fp32 == 600 // 32
    with mf.matmul_precision("bf16"):
        bf16 = mf._split_for(768, 128, 9600)
    assert bf16 == 600 // 16 and bf16 > fp32
    assert mf._split_for(24, 40, 300000) == 512         # skinny: capped at 512 slabs
    for M, N, K in ((768, 768, 9600), (64, 792, 614400), (2304, 768, 9600)):
        s = mf._split_for(M, N, K)
        assert 1 <= s <= 512 and K / s >= 512 - 16


def test_split_k_wave_quantisation_fp32():
    """fp32 split factors by wave quantisation (functional._split_fill, round 5;
    profiles/round5/split_study.txt): tiles x split workgroups fill whole rounds of one per CU,
    384-512 tiles stay unsplit, narrow outputs keep their deep splits, bf16 keeps the round-4
    rule."""
    from mdemi import functional as mf
    assert mf._split_for(768, 768, 9600) == 7        # 36 tiles x 7 = 252 workgroups (was 18: 648)
    assert mf._split_for(384, 1536, 38400) == 7      # 36 tiles (was 28)
    assert mf._split_for(2304, 768, 9600) == 7       # 108 tiles x 7 = 756 = 3 full rounds
    assert mf._split_for(9600, 768, 3072) == 1       # 450 tiles: one round at two workgroups per CU
    assert 2 <= mf._split_for(6144, 1536, 2400) <= 4  # 576 tiles: 2.25 rounds unsplit
    assert mf._split_for(576, 192, 153600) == 102    # 10 tiles: the deep split stays
    prev = mf._SPLIT_POLICY
    try:
        mf._SPLIT_POLICY = "legacy"
        assert mf._split_for(768, 768, 9600) == 18
    finally:
        mf._SPLIT_POLICY = prev
    with mf.matmul_precision("bf16"):
        assert mf._split_for(768, 768, 9600) == 28   # the round-4 rule: 1024 // 36
