"""utils/common_utils.py pieces on the hot path: parse() reads the reference's
JSON configs unchanged (common_utils.py:34-52); gpu_ids select devices through
HIP_VISIBLE_DEVICES (ROCm's CUDA_VISIBLE_DEVICES).  RunningAverage /
RunningAverageDict (common_utils.py:92-135) accumulate the eval metrics.
save_checkpoint (common_utils.py:12-31) writes the reference's training-state file;
load_checkpoint reads one (the reference's or ours) back for a resume."""
import json
import os
from collections import OrderedDict

import torch

CHECKPOINT_KEYS = ("epoch", "iter", "best_epoch", "best_iter", "model_state_dict", "optimizer_state_dict", "best")


def _unwrap(model):
    # the reference unwraps DistributedDataParallel (common_utils.py:19-20); mdemi's data
    # parallelism (train.ddp.GradAllReduce) never wraps the model, any .module wrapper is peeled
    while hasattr(model, "module") and isinstance(model.module, torch.nn.Module):
        model = model.module
    return model


def save_checkpoint(prefix: str, model, optimizer, current_epoch, current_iter, best_value, save_dir: str,
                    best_epoch=None, best_iter=None, *, model_only: bool = False) -> None:
    """common_utils.py:12-31: ``{save_dir}/{prefix}.pth`` holding epoch, iter, best_epoch /
    best_iter (default: the current ones), the model's state_dict, the optimizer's
    state_dict (None with model_only) and best.  FusedAdamW.state_dict() is torch.optim.AdamW's
    layout (per-parameter "step", params index lists), so the file loads into the reference's
    torch AdamW and back."""
    model = _unwrap(model)
    torch.save({
        "epoch": current_epoch,
        "iter": current_iter,
        "best_epoch": best_epoch if best_epoch is not None else current_epoch,
        "best_iter": best_iter if best_iter is not None else current_iter,
        "model_state_dict": model.state_dict(),
        "optimizer_state_dict": optimizer.state_dict() if not model_only else None,
        "best": best_value,
    }, f"{save_dir}/{prefix}.pth")


def load_checkpoint(path: str, model=None, optimizer=None, map_location="cpu", strict: bool = True) -> dict:
    """Read a save_checkpoint file (weights_only: nothing in it is executed) and, when given,
    load its model state (strict) and optimizer state into ``model`` / ``optimizer``.
    Returns the file's dict (epoch, iter, best_epoch, best_iter, best, ...).  Raises
    ValueError on a file that is not a training-state checkpoint, or when an optimizer is
    given but the file was saved model_only."""
    ck = torch.load(path, map_location=map_location, weights_only=True)
    if not isinstance(ck, dict) or "model_state_dict" not in ck:
        raise ValueError(f"{path}: not a save_checkpoint file (keys {sorted(ck)[:8] if isinstance(ck, dict) else type(ck)})")
    if model is not None:
        _unwrap(model).load_state_dict(ck["model_state_dict"], strict=strict)
    if optimizer is not None:
        if ck.get("optimizer_state_dict") is None:
            raise ValueError(f"{path} was saved model_only: no optimizer state to resume from")
        optimizer.load_state_dict(ck["optimizer_state_dict"])
    return ck


def parse(json_path: str, write_option: bool = True) -> dict:
    with open(json_path, "r", encoding="utf-8") as f:
        opt = json.load(f, object_pairs_hook=OrderedDict)
    gpu_list = ",".join(str(x) for x in opt["gpu_ids"])
    os.environ["HIP_VISIBLE_DEVICES"] = gpu_list
    opt["num_gpus"] = len(opt["gpu_ids"])
    print("export HIP_VISIBLE_DEVICES=" + gpu_list)
    print("number of GPUs=" + str(opt["num_gpus"]))
    if write_option:
        os.makedirs(opt["output_dir"], exist_ok=True)
        with open(os.path.join(opt["output_dir"], "option.json"), "w", encoding="utf-8") as f:
            json.dump(opt, f, indent="\t")
    return opt


class RunningAverage:
    """common_utils.py:92-113: incremental mean; tensors are read with .item()."""

    def __init__(self):
        self._avg = 0.0
        self._count = 0

    def append(self, value) -> None:
        if hasattr(value, "item"):
            value = value.item()
        self._avg = (value + self._count * self._avg) / (self._count + 1)
        self._count += 1

    @property
    def avg(self) -> float:
        return self._avg

    @property
    def count(self) -> int:
        return self._count

    def reset(self) -> None:
        self._avg = 0.0
        self._count = 0


class RunningAverageDict:
    """common_utils.py:116-135: one RunningAverage per key of the first dict seen."""

    def __init__(self):
        self._dict = None

    def update(self, new_dict) -> None:
        if self._dict is None:
            self._dict = {k: RunningAverage() for k in new_dict}
        for k, v in new_dict.items():
            self._dict[k].append(v)

    def get_value(self) -> dict:
        return {k: v.avg for k, v in self._dict.items()}

    def reset(self) -> None:
        if self._dict is None:
            return
        for v in self._dict.values():
            v.reset()
