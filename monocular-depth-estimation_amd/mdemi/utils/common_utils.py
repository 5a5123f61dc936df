"""utils/common_utils.py pieces on the hot path: parse() reads the reference's
JSON configs unchanged (common_utils.py:34-52); gpu_ids select devices through
HIP_VISIBLE_DEVICES (ROCm's CUDA_VISIBLE_DEVICES).  RunningAverage /
RunningAverageDict (common_utils.py:92-135) accumulate the eval metrics."""
import json
import os
from collections import OrderedDict


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
