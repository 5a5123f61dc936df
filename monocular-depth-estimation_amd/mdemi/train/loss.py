"""SILog loss (restated; config keys loss.alpha / loss.beta / loss.per_image).
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
