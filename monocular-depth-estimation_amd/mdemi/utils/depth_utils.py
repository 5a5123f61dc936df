"""utils/depth_utils.py surface: cal_eval_mask and tcompute_errors with the
reference's semantics (numpy, per image), plus the GPU path the evaluation
loop uses at dataset scale: the crop is a rectangle, so `eval_crop_rect`
computes it with the reference's formulas and `tcompute_errors_gpu` reduces
the 9 metrics for a whole batch in one libmdemi launch pair
(mdemi_depth_metrics: per-image fixed-order sums, fp64 finalize)."""
import numpy as np

__all__ = ["cal_eval_mask", "tcompute_errors", "eval_crop_rect", "tcompute_errors_gpu", "METRICS"]

METRICS = ("a1", "a2", "a3", "abs_rel", "sq_rel", "rmse", "rmse_log", "silog", "log_10")


def eval_crop_rect(opt, gt_height, gt_width, data_type: str):
    """(y0, y1, x0, x1) of the evaluation crop (depth_utils.py:4-29)."""
    if opt["garg_crop"]:
        return (int(0.40810811 * gt_height), int(0.99189189 * gt_height),
                int(0.03594771 * gt_width), int(0.96405229 * gt_width))
    if opt["eigen_crop"]:
        if data_type in ("KITTI", "ONLINE"):
            return (int(0.3324324 * gt_height), int(0.91351351 * gt_height),
                    int(0.0359477 * gt_width), int(0.96405229 * gt_width))
        if data_type == "NYU":
            return (45, 471, 41, 601)
        raise ValueError(f"Unsupported data_type {data_type}.")
    raise ValueError("Unsupported crop configuration.")


def cal_eval_mask(opt, gt_depth, data_type: str):
    gh, gw = gt_depth.shape[-2:]
    y0, y1, x0, x1 = eval_crop_rect(opt, gh, gw, data_type)
    mask = np.zeros(gt_depth.shape[-2:], dtype=bool)
    mask[y0:y1, x0:x1] = True
    return mask


def tcompute_errors(gt: np.ndarray, pred: np.ndarray) -> dict:
    """The reference's 9 metrics on already-masked 1-D arrays (depth_utils.py:32-54)."""
    thresh = np.maximum(gt / pred, pred / gt)
    err = np.log(pred) - np.log(gt)
    return dict(a1=(thresh < 1.25).mean(), a2=(thresh < 1.25 ** 2).mean(), a3=(thresh < 1.25 ** 3).mean(),
                abs_rel=np.mean(np.abs(gt - pred) / gt), sq_rel=np.mean(((gt - pred) ** 2) / gt),
                rmse=np.sqrt(((gt - pred) ** 2).mean()),
                rmse_log=np.sqrt(((np.log(gt) - np.log(pred)) ** 2).mean()),
                silog=np.sqrt(np.mean(err ** 2) - np.mean(err) ** 2) * 100,
                log_10=(np.abs(np.log10(gt) - np.log10(pred))).mean())


def tcompute_errors_gpu(pred, gt, eval_opt, data_type, clamp_pred=True):
    """Per-image metrics for a batch on the GPU: pred/gt (B, 1, H, W) fp32 CUDA tensors; valid =
    crop & min_depth_eval < gt < max_depth_eval (cfg eval.*).  Returns a list of dicts (one per
    image, the reference's keys) -- feed them to RunningAverageDict / all_reduce_dict."""
    from .. import functional as mf
    h, w = gt.shape[-2:]
    rect = eval_crop_rect(eval_opt, h, w, data_type)
    out = mf.depth_metrics(pred, gt, rect, eval_opt["min_depth_eval"], eval_opt["max_depth_eval"],
                           clamp_pred=clamp_pred).cpu().numpy()
    return [dict(zip(METRICS, row[:9].tolist())) for row in out]
