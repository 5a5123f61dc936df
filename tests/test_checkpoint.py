"""CPU checks of checkpoint interop (mdemi.utils.checkpoint), modelled on the
reference's loader (model/NewCRFs/newcrf_utils.py:73-264) and its rename
scripts (checkpoint/*_rename.py).  No GPU: models are constructed on the host
and only their parameters are compared."""
from collections import OrderedDict

import pytest
import torch
import torch.nn.functional as F

from mdemi.model.NewCRFs import NewCRFDepth
from mdemi.model.NewCRFs.swin_transformer import SwinTransformer
from mdemi.utils import checkpoint as ck


def _tiny_swin(window=7):
    return SwinTransformer(embed_dim=96, depths=[2, 2, 6, 2], num_heads=[3, 6, 12, 24], window_size=window,
                           ape=False, drop_path_rate=0.0, patch_norm=True)


def _randomised(model, seed):
    g = torch.Generator().manual_seed(seed)
    return OrderedDict((k, torch.randn(v.shape, generator=g).to(v.dtype) if v.is_floating_point() else v.clone())
                       for k, v in model.state_dict().items())


@pytest.mark.parametrize("wrap", ["model", "state_dict", "bare"])
def test_load_checkpoint_prefix_and_container(tmp_path, wrap):
    src = _randomised(_tiny_swin(), 1)
    sd = OrderedDict(("module." + k, v) for k, v in src.items())
    obj = {"model": sd} if wrap == "model" else {"state_dict": sd} if wrap == "state_dict" else sd
    path = tmp_path / "ckpt.pth"
    torch.save(obj, path)
    dst = _tiny_swin()
    ck.load_checkpoint(dst, str(path), strict=True)
    for k, v in dst.state_dict().items():
        assert torch.equal(v, src[k]), k


def test_moby_encoder_branch(tmp_path):
    src = _randomised(_tiny_swin(), 2)
    sd = {"encoder." + k: v for k, v in src.items()}
    sd.update({"encoder_k." + k: torch.zeros_like(v) for k, v in src.items()})
    dst = _tiny_swin()
    ck.load_checkpoint(dst, {"model": sd}, strict=True)
    for k, v in dst.state_dict().items():
        assert torch.equal(v, src[k]), k


def test_rel_pos_bias_table_resized_bicubic():
    # a window-12 checkpoint (23*23 rows) into a window-7 backbone (13*13 rows)
    big = _randomised(_tiny_swin(12), 3)
    dst = _tiny_swin(7)
    err = ck.load_state_dict(dst, {}, strict=False)  # everything missing: reported, not raised
    assert err
    sd = {k: v for k, v in big.items() if "relative_position_index" not in k and "attn_mask" not in k}
    ck.load_checkpoint(dst, sd, strict=False)
    key = "layers.0.blocks.0.attn.relative_position_bias_table"
    t = big[key]
    want = F.interpolate(t.permute(1, 0).reshape(1, t.shape[1], 23, 23), size=(13, 13), mode="bicubic")
    want = want.reshape(t.shape[1], 169).permute(1, 0)
    assert torch.allclose(dst.state_dict()[key], want, atol=0, rtol=0)
    # bicubic keeps a constant table constant
    c = torch.full((23 * 23, 4), 0.37)
    assert torch.allclose(ck.resize_rel_pos_bias_table(c, 169), torch.full((169, 4), 0.37), atol=1e-6)
    # other parameters of matching shape load unchanged
    assert torch.equal(dst.state_dict()["patch_embed.proj.weight"], big["patch_embed.proj.weight"])


def test_head_count_mismatch_passes_table(capsys):
    dst = _tiny_swin()
    key = "layers.0.blocks.0.attn.relative_position_bias_table"
    before = dst.state_dict()[key].clone()
    sd = {key: torch.randn(169, 5)}
    ck.load_checkpoint(dst, sd, strict=False)
    assert torch.equal(dst.state_dict()[key], before)
    assert f"Error in loading {key}, pass" in capsys.readouterr().out


def test_strict_mismatch_raises():
    dst = _tiny_swin()
    sd = dict(dst.state_dict())
    sd["not_a_param"] = torch.zeros(1)
    with pytest.raises(RuntimeError, match="unexpected key"):
        ck.load_state_dict(dst, sd, strict=True)
    sd.pop("not_a_param")
    sd.pop("norm0.weight")
    with pytest.raises(RuntimeError, match="missing keys"):
        ck.load_state_dict(dst, sd, strict=True)


def test_non_file_raises(tmp_path):
    with pytest.raises(IOError):
        ck.load_checkpoint(_tiny_swin(), str(tmp_path / "absent.pth"))


def test_newcrfdepth_pretrained_backbone(tmp_path):
    src = _randomised(_tiny_swin(), 4)
    path = tmp_path / "swin_tiny.pth"
    torch.save({"model": src}, path)
    m = NewCRFDepth(version="tiny07", max_depth=10.0, pretrained=str(path))
    for k, v in m.backbone.state_dict().items():
        assert torch.equal(v, src[k]), k


def test_rename_scripts():
    old = {"model": OrderedDict([("module.backbone.x", torch.ones(1)),
                                 ("module.encoder.original_model.bn2.weight", torch.ones(2)),
                                 ("module.decoder.y", torch.zeros(1))])}
    n = ck.rename_newcrfs_checkpoint(old)["model"]
    assert list(n) == ["backbone.x", "encoder.original_model.bn2.weight", "decoder.y"]
    a = ck.rename_adabins_checkpoint(old)["model"]
    assert list(a) == ["backbone.x", "decoder.y"]
