"""utils/common_utils.py pieces on the hot path: parse() reads the reference's
JSON configs unchanged (common_utils.py:34-52); gpu_ids select devices through
HIP_VISIBLE_DEVICES (ROCm's CUDA_VISIBLE_DEVICES)."""
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
