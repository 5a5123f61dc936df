"""Checkpoint interop: load upstream NeW-CRFs / AdaBins / Swin weights into the
mdemi model mirrors.

Restates the reference's loader semantics:
  * `load_checkpoint` -- model/NewCRFs/newcrf_utils.py:194-264: take
    'state_dict' / 'model' / the bare dict, strip a leading 'module.' prefix,
    keep only the 'encoder.' branch of MoBY checkpoints, reshape
    `absolute_pos_embed` (N, L, C) -> (N, C, H, W), and bicubically resize every
    `relative_position_bias_table` whose window size differs (e.g. the
    window-12 ImageNet-22k Swin-L loaded into the window-7 "large07"
    backbone: (23*23, nH) -> (13*13, nH)).
  * `load_state_dict` -- newcrf_utils.py:73-138: non-strict by default; missing
    keys (ignoring BN `num_batches_tracked`), unexpected keys and shape
    mismatches are collected, reported on rank 0, and raised when strict.
  * `rename_newcrfs_checkpoint` / `rename_adabins_checkpoint` --
    checkpoint/newcrfs_checkpoint_rename.py:10-15,
    checkpoint/adabins_checkpoint_rename.py:10-18: the upstream release
    checkpoints' key rewrite ('module.' dropped; AdaBins also drops the unused
    `encoder.original_model.bn2.*`).

Files are read with `torch.load(..., weights_only=True)` only: nothing in a
checkpoint file is executed.  This is host-side plumbing run once at model
construction, not part of the measured path; tensors are copied into the
model's existing (device) parameters by `nn.Module._load_from_state_dict`.
"""
import os
from collections import OrderedDict

import torch
import torch.nn.functional as F
from torch import nn

__all__ = ["load_checkpoint", "load_state_dict", "load_backbone_checkpoint", "read_checkpoint",
           "rename_newcrfs_checkpoint", "rename_adabins_checkpoint", "resize_rel_pos_bias_table"]


def _rank0():
    import torch.distributed as dist
    return not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0


def read_checkpoint(filename, map_location="cpu"):
    """newcrf_utils.py:167-191 for local files (no modelzoo/URL schemes: there is no network)."""
    if not os.path.isfile(filename):
        raise IOError(f"{filename} is not a checkpoint file")
    return torch.load(filename, map_location=map_location, weights_only=True)


def load_state_dict(module, state_dict, strict=False, logger=None):
    """newcrf_utils.py:73-138.  Returns the error message list (empty on an exact match)."""
    unexpected, missing_all, err = [], [], []
    metadata = getattr(state_dict, "_metadata", None)
    state_dict = OrderedDict(state_dict)
    if metadata is not None:
        state_dict._metadata = metadata

    def load(m, prefix=""):
        if isinstance(m, (nn.DataParallel, nn.parallel.DistributedDataParallel)):
            m = m.module
        local = {} if metadata is None else metadata.get(prefix[:-1], {})
        m._load_from_state_dict(state_dict, prefix, local, True, missing_all, unexpected, err)
        for name, child in m._modules.items():
            if child is not None:
                load(child, prefix + name + ".")

    load(module)
    missing = [k for k in missing_all if "num_batches_tracked" not in k]
    if unexpected:
        err.append(f"unexpected key in source state_dict: {', '.join(unexpected)}\n")
    if missing:
        err.append(f"missing keys in source state_dict: {', '.join(missing)}\n")
    if err and _rank0():
        msg = "\n".join(["The model and loaded state dict do not match exactly\n"] + err)
        if strict:
            raise RuntimeError(msg)
        if logger is not None:
            logger.warning(msg)
        else:
            print(msg)
    return err


def resize_rel_pos_bias_table(table, L2):
    """(L1, nH) -> (L2, nH) by bicubic resampling of the (S1, S1) bias grid per head
    (newcrf_utils.py:245-260; align_corners=False, as F.interpolate's default there)."""
    L1, nH = table.shape
    if L1 == L2:
        return table
    S1, S2 = int(L1 ** 0.5), int(L2 ** 0.5)
    grid = table.permute(1, 0).reshape(1, nH, S1, S1)
    out = F.interpolate(grid.float(), size=(S2, S2), mode="bicubic")
    return out.reshape(nH, L2).permute(1, 0).to(table.dtype)


def _extract(checkpoint, filename):
    if not isinstance(checkpoint, dict):
        raise RuntimeError(f"No state_dict found in checkpoint file {filename}")
    if "state_dict" in checkpoint:
        return checkpoint["state_dict"]
    if "model" in checkpoint:
        return checkpoint["model"]
    return checkpoint


def load_checkpoint(model, filename, map_location="cpu", strict=False, logger=None):
    """newcrf_utils.py:194-264.  `filename` may also be an already-loaded dict."""
    checkpoint = filename if isinstance(filename, dict) else read_checkpoint(filename, map_location)
    state_dict = _extract(checkpoint, filename if isinstance(filename, str) else "<dict>")
    if list(state_dict.keys())[0].startswith("module."):
        state_dict = {k[7:]: v for k, v in state_dict.items()}
    if sorted(state_dict.keys())[0].startswith("encoder"):  # MoBY: online branch only
        state_dict = {k.replace("encoder.", ""): v for k, v in state_dict.items() if k.startswith("encoder.")}
    state_dict = dict(state_dict)

    ape = state_dict.get("absolute_pos_embed")
    if ape is not None:
        cur = getattr(model, "absolute_pos_embed", None)
        if cur is None:
            msg = "Error in loading absolute_pos_embed, pass"
            logger.warning(msg) if logger is not None else print(msg)
        else:
            N1, L, C1 = ape.shape
            N2, C2, H, W = cur.shape
            if N1 != N2 or C1 != C2 or L != H * W:
                msg = "Error in loading absolute_pos_embed, pass"
                logger.warning(msg) if logger is not None else print(msg)
            else:
                state_dict["absolute_pos_embed"] = ape.view(N2, H, W, C2).permute(0, 3, 1, 2)

    current = model.state_dict()
    for key in [k for k in state_dict if "relative_position_bias_table" in k]:
        if key not in current:
            continue
        L1, nH1 = state_dict[key].shape
        L2, nH2 = current[key].shape
        if nH1 != nH2:
            msg = f"Error in loading {key}, pass"
            logger.warning(msg) if logger is not None else print(msg)
        elif L1 != L2:
            state_dict[key] = resize_rel_pos_bias_table(state_dict[key], L2)

    load_state_dict(model, state_dict, strict, logger)
    return checkpoint


def load_backbone_checkpoint(backbone, pretrained):
    """SwinTransformer.init_weights(pretrained=str) (swin_transformer.py:584): non-strict load."""
    return load_checkpoint(backbone, pretrained, strict=False)


def rename_newcrfs_checkpoint(old):
    """checkpoint/newcrfs_checkpoint_rename.py: {'model': {k without 'module.': v}}."""
    new = OrderedDict(model=OrderedDict())
    for k, v in old["model"].items():
        new["model"][k.replace("module.", "")] = v
    return new


def rename_adabins_checkpoint(old):
    """checkpoint/adabins_checkpoint_rename.py: as NeW-CRFs, minus encoder.original_model.bn2.*
    (the timm head BN that UnetAdaptiveBins' encoder never runs)."""
    new = OrderedDict(model=OrderedDict())
    for k, v in old["model"].items():
        nk = k.replace("module.", "")
        if "encoder.original_model.bn2" in nk:
            continue
        new["model"][nk] = v
    return new
