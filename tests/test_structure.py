"""CPU checks of the drop-in boundary: the mdemi model mirrors expose the
reference's state_dict (same keys, shapes, dtypes and order — the order also
drives the closed-form weight fill) and the C-ABI library exports every
symbol include/mdemi.h and include/mdemi_ext.h declare."""
import os
import re

import pytest

from golden_util import Golden, spec_of

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol():
    from mdemi import _lib
    lib = _lib.load()
    header = "".join(open(h).read() for h in _lib.HEADER_PATHS)
    declared = set(re.findall(r"\b(mdemi_[a-z0-9_]+)\s*\(", header))
    assert len(declared) > 30
    for name in sorted(declared):
        assert hasattr(lib, name), f"libmdemi.so does not export {name}"
    # and the ctypes table covers the header
    assert declared <= set(_lib.exported_symbols()), declared - set(_lib.exported_symbols())


def test_library_version_and_error_path():
    from mdemi import _lib
    lib = _lib.load()
    assert lib.mdemi_version() >= 1
    # an invalid call fails with a negative code and a message, without touching the GPU
    rc = lib.mdemi_layernorm_fwd(None, None, None, None, None, None, 0, 0, 1e-5, None)
    assert rc < 0
    assert b"layernorm" in lib.mdemi_last_error()
    with pytest.raises(RuntimeError):
        _lib.check(rc, "layernorm_fwd")


def _spec_eq(model, golden_name):
    want = Golden(golden_name).spec
    got = spec_of(model)
    assert [k for k, _, _ in got] == [k for k, _, _ in want]
    assert got == want


def test_state_dict_matches_reference_newcrfs_tiny07():
    from mdemi.model.NewCRFs import NewCRFDepth
    _spec_eq(NewCRFDepth(version="tiny07", max_depth=10.0), "newcrfs_tiny07")


def test_state_dict_matches_reference_modules():
    import torch.nn as nn
    from mdemi.model.NewCRFs.newcrf_layers import NewCRF
    from mdemi.model.NewCRFs.swin_transformer import BasicLayer, PatchMerging, SwinTransformer
    from mdemi.model.NewCRFs.uper_crf_head import PSP
    from mdemi.model.NewCRFs.NewCRFDepth import DispHead
    _spec_eq(BasicLayer(dim=64, depth=2, num_heads=2, window_size=7, downsample=PatchMerging),
             "swin_basic_layer_10x12")
    _spec_eq(SwinTransformer(embed_dim=64, depths=[2, 2, 2, 2], num_heads=[2, 4, 8, 16], window_size=7,
                             drop_path_rate=0.0), "swin_backbone")
    _spec_eq(NewCRF(input_dim=96, embed_dim=128, window_size=7, v_dim=64, num_heads=4), "newcrf_layer")
    _spec_eq(PSP(in_channels=[16, 32, 64, 128], in_index=[0, 1, 2, 3], pool_scales=(1, 2, 3, 6), channels=512,
                 dropout_ratio=0.0, num_classes=32, norm_cfg=dict(type="BN", requires_grad=True),
                 align_corners=False), "psp_head")
    _spec_eq(DispHead(input_dim=128), "disp_head")
    del nn


def test_large07_parameter_count():
    """NewCRFs large07 = 270,444,877 params (backbone 194,998,164)."""
    from mdemi.model.NewCRFs import NewCRFDepth
    m = NewCRFDepth(version="large07", max_depth=10.0)
    assert sum(p.numel() for p in m.parameters()) == 270_444_877
    assert sum(p.numel() for p in m.backbone.parameters()) == 194_998_164


def _fake_backend():
    import torch.nn as nn
    m = nn.Module()
    m.conv_stem, m.bn1, m.act1 = nn.Identity(), nn.Identity(), nn.Identity()
    m.blocks = nn.Sequential(*[nn.Identity() for _ in range(7)])
    m.conv_head, m.act2 = nn.Identity(), nn.Identity()
    return m


def test_state_dict_matches_reference_adabins():
    from mdemi.model.Adabins import UnetAdaptiveBins, mViT
    _spec_eq(UnetAdaptiveBins(_fake_backend(), n_bins=256, min_val=1e-3, max_val=10.0), "adabins_head")
    _spec_eq(mViT(128, n_query_channels=128, patch_size=16, dim_out=256, embedding_dim=128, norm="linear"), "mvit")


def test_adabins_parameter_counts():
    """AdaBins non-encoder params 49,916,544; EfficientNet-B5 28.34 M incl. conv_head."""
    from mdemi.model.Adabins import UnetAdaptiveBins
    m = UnetAdaptiveBins.build(256, 1e-3, 10.0)
    enc = sum(p.numel() for p in m.encoder.parameters())
    assert sum(p.numel() for p in m.parameters()) - enc == 49_916_544
    assert enc == 28_336_688
    keys = list(m.state_dict().keys())
    assert keys[0] == "encoder.original_model.conv_stem.weight"
    assert "encoder.original_model.blocks.6.2.se.conv_expand.bias" in keys


DFV8_GOLDEN_OPT = {"hidden_dim": 64, "num_heads": 4, "num_bins": 32, "num_aux": 16, "img_size": [64, 96],
                   "attn_drop_prob": 0.0, "drop_prob": 0.0}


def test_state_dict_matches_reference_depthformer_v8():
    from mdemi.model.Depthformer import DepthformerV8
    _spec_eq(DepthformerV8(_fake_backend(), DFV8_GOLDEN_OPT, min_depth=1e-3, max_depth=10.0), "depthformer_v8")


def test_depthformer_v8_parameter_counts():
    """Depthformer v8 decoder params 7,167,296 (hidden 256, 4 heads, 256 bins/aux)."""
    from mdemi.model.Depthformer import DepthformerV8
    opt = {"hidden_dim": 256, "num_heads": 4, "num_bins": 256, "num_aux": 256, "img_size": [352, 1216]}
    m = DepthformerV8.build(opt, 1e-3, 80.0)
    assert sum(p.numel() for p in m.decoder.parameters()) == 7_167_296
    assert sum(p.numel() for p in m.encoder.parameters()) == 27_288_112  # B5 without conv_head/bn2
