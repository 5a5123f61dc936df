"""CPU restatement of utils/depth_utils.py (evaluation crop + 9 depth metrics)
and the restated SILog loss.  TEST INFRASTRUCTURE ONLY — see oracle/__init__.py.
depth metrics pinned by tests/golden/depth_metrics.npz; SILog parity unpinned
(the reference's loss module is absent from the snapshot).
"""
import numpy as np
import torch


def cal_eval_mask(opt, gt_depth, data_type):  # depth_utils.py:4-29
    gh, gw = gt_depth.shape[-2:]
    m = np.zeros(gt_depth.shape[-2:], dtype=bool)
    if opt["garg_crop"]:
        m[int(0.40810811 * gh):int(0.99189189 * gh), int(0.03594771 * gw):int(0.96405229 * gw)] = True
    elif opt["eigen_crop"]:
        if data_type in ("KITTI", "ONLINE"):
            m[int(0.3324324 * gh):int(0.91351351 * gh), int(0.0359477 * gw):int(0.96405229 * gw)] = True
        elif data_type == "NYU":
            m[45:471, 41:601] = True
        else:
            raise ValueError(f"Unsupported data_type {data_type}.")
    else:
        raise ValueError("Unsupported crop configuration.")
    return m


def compute_errors(gt, pred):  # depth_utils.py:32-54
    thresh = np.maximum(gt / pred, pred / gt)
    err = np.log(pred) - np.log(gt)
    return dict(
        a1=(thresh < 1.25).mean(), a2=(thresh < 1.25 ** 2).mean(), a3=(thresh < 1.25 ** 3).mean(),
        abs_rel=np.mean(np.abs(gt - pred) / gt), sq_rel=np.mean(((gt - pred) ** 2) / gt),
        rmse=np.sqrt(((gt - pred) ** 2).mean()), rmse_log=np.sqrt(((np.log(gt) - np.log(pred)) ** 2).mean()),
        silog=np.sqrt(np.mean(err ** 2) - np.mean(err) ** 2) * 100,
        log_10=(np.abs(np.log10(gt) - np.log10(pred))).mean())


def silog_loss(pred, gt, min_depth=1e-3, alpha=10.0, beta=0.15, per_image=False, unbiased=False):
    """alpha*sqrt(Var(g) + beta*mean(g)^2), g = log pred - log gt on gt > min_depth (restated, unpinned)."""

    def group(p, g):
        m = g > min_depth
        d = torch.log(p[m]) - torch.log(g[m])
        var = d.var() if unbiased else (d * d).mean() - d.mean() ** 2
        return alpha * torch.sqrt(var + beta * d.mean() ** 2)

    if per_image:
        return torch.stack([group(pred[b], gt[b]) for b in range(pred.shape[0])]).mean()
    return group(pred, gt)
