"""SILog loss (restated; config keys loss.alpha / loss.beta / loss.per_image) and
the AdaBins bin chamfer loss (config key loss.chamfer_weight; restated from
upstream AdaBins' BinsChamferLoss -- the reference's loss module is absent).
AdaBins / Depthformer predictions are at half resolution and are resized to
the ground truth with bilinear align_corners=True first (upstream AdaBins
convention; parity unpinned)."""
import torch.nn as nn

from .. import functional as mf


class SILogLoss(nn.Module):
    def __init__(self, alpha=10.0, beta=0.15, per_image=False, min_depth=1e-3, unbiased=False):
        super().__init__()
        self.alpha, self.beta, self.per_image = float(alpha), float(beta), bool(per_image)
        self.min_depth, self.unbiased = float(min_depth), bool(unbiased)

    def forward(self, pred, gt):
        """pred (B,1,h,w), gt (B,1,H,W) NCHW (C=1, so also NHWC)."""
        if pred.shape[-2:] != gt.shape[-2:]:
            B, _, h, w = pred.shape
            pred = mf.interpolate_bilinear(pred.reshape(B, h, w, 1), size=tuple(gt.shape[-2:]),
                                           align_corners=True).reshape(B, 1, *gt.shape[-2:])
        return mf.silog_loss(pred, gt, self.min_depth, self.alpha, self.beta, self.per_image, self.unbiased)


class BinsChamferLoss(nn.Module):
    """Chamfer distance between each image's bin centres and its valid (>= 1e-3) GT depths:
    mean over centres of the squared distance to the nearest depth plus mean over depths of
    the squared distance to the nearest centre, averaged over the batch (one libmdemi sweep
    forward, one backward)."""

    def __init__(self, thresh=1e-3, from_edges=True):
        super().__init__()
        self.thresh, self.from_edges = float(thresh), bool(from_edges)

    def forward(self, bins, gt):
        """bins: edges (B, P+1) (AdaBins), or centres (B, P, 1, 1) with from_edges=False
        (Depthformer v8)."""
        return mf.bins_chamfer(bins, gt, self.thresh, self.from_edges)
