"""Evaluation path on the GPU: inference, flip-eval, the
9 depth metrics and their cross-rank mean.

The reference's driver (run.py) is absent from the snapshot; what it did is
fixed by the config keys eval.{min_depth_eval, max_depth_eval, garg_crop,
eigen_crop, flip_eval} (json/{nyu,kitti}/*.json) and by the helpers it
called: cal_eval_mask + tcompute_errors (utils/depth_utils.py:4-54),
RunningAverageDict (utils/common_utils.py:92-135) and
all_reduce_dict(op="mean") (utils/dist_utils.py:67-76).  Restated here (parity
of the driver itself is unpinned; each helper is pinned by its own tests):

  pred = model(img)                       # depth, NCHW
  if flip_eval: pred = (pred + flip_w(model(flip_w(img)))) / 2
  pred -> GT resolution (bilinear, align_corners=True) when the model
          predicts at half resolution (AdaBins / Depthformer v8)
  per image: metrics over crop & min_depth_eval < gt < max_depth_eval,
             pred clamped into [min_depth_eval, max_depth_eval]

Every step is a libmdemi launch (flip: mdemi_flip_w / mdemi_flip_avg_w;
resize: mdemi_bilinear_*; metrics: mdemi_depth_metrics); only the per-image
metric rows (B x 10 fp64) come back to the host.
"""

import torch

from . import functional as mf
from .utils.common_utils import RunningAverageDict
from .utils.depth_utils import tcompute_errors_gpu
from .utils.dist_utils import all_reduce_dict

__all__ = ["predict_depth", "evaluate_batch", "evaluate", "GraphedPredictor"]


def _depth_of(out):
    # NewCRFDepth -> depth; UnetAdaptiveBins -> (pred, bin_edges); DepthformerV8 -> (depth, centers, attn)
    return out[0] if isinstance(out, (tuple, list)) else out


def predict_depth(model, img, flip_eval=False, size=None):
    """Depth (B,1,H,W) for an NCHW image batch; flip-eval averages in the flipped pass; `size`
    resizes the prediction (bilinear, align_corners=True) to the ground-truth resolution."""
    with torch.no_grad():
        pred = _depth_of(model(img))
        if flip_eval:
            pred = mf.flip_avg_w(pred, _depth_of(model(mf.flip_w(img))))
        if size is not None and tuple(pred.shape[-2:]) != tuple(size):
            B, _, h, w = pred.shape
            pred = mf.interpolate_bilinear(pred.reshape(B, h, w, 1), size=tuple(size),
                                           align_corners=True).reshape(B, 1, *size)
    return pred


def evaluate_batch(model, img, gt, eval_opt, data_type):
    """Per-image metric dicts (the reference's keys) for one batch.  `model` may be a
    GraphedPredictor (its capture fixes flip_eval)."""
    if isinstance(model, GraphedPredictor):
        pred = model(img)
        if tuple(pred.shape[-2:]) != tuple(gt.shape[-2:]):
            B, _, h, w = pred.shape
            pred = mf.interpolate_bilinear(pred.reshape(B, h, w, 1), size=tuple(gt.shape[-2:]),
                                           align_corners=True).reshape(B, 1, *gt.shape[-2:])
    else:
        pred = predict_depth(model, img, bool(eval_opt.get("flip_eval", False)), size=tuple(gt.shape[-2:]))
    return tcompute_errors_gpu(pred, gt, eval_opt, data_type)


class GraphedPredictor:
    """Inference (model forward, + the flipped pass and average when flip_eval) captured once into
    a hipGraph (torch.cuda.CUDAGraph) for a fixed input shape and replayed per batch: one graph
    launch instead of ~1000 kernel launches.  Every kernel is a libmdemi launch on the capturing
    stream; workspaces come from torch's allocator (the graph's private pool) and nothing on the
    path synchronises with the host.  Eval mode only: no dropout / drop-path seeds are baked in.
    Warm-up runs happen before capture so the GEMM autotuner has settled on every shape."""

    def __init__(self, model, example_img, flip_eval=False, warmup=2):
        if model.training:
            raise ValueError("GraphedPredictor needs model.eval() (training draws host-side RNG seeds)")
        self.model, self.flip_eval = model, bool(flip_eval)
        self.static_in = example_img.detach().clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                predict_depth(model, self.static_in, self.flip_eval)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        from .train.builder import quiesce_process_group
        quiesce_process_group()  # no eager collective may be polled by the watchdog mid-capture
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.static_out = predict_depth(model, self.static_in, self.flip_eval)

    def __call__(self, img):
        if img.shape != self.static_in.shape:
            raise ValueError(f"GraphedPredictor captured {tuple(self.static_in.shape)}, got {tuple(img.shape)}")
        self.static_in.copy_(img)
        self.graph.replay()
        return self.static_out.clone()


def evaluate(model, batches, eval_opt, data_type, weight_by_count=False):
    """Running mean of the metrics over (img, gt) batches on this rank, then the mean over ranks
    (all_reduce_dict op="mean"; a pass-through without a process group).

    The rank mean is unweighted, as all_reduce_dict(op="mean") makes it: exact when every
    rank sees the same number of images (a padded DistributedSampler).  weight_by_count=True
    instead reduces (sum, count) per metric and divides once -- the exact dataset mean when
    ranks see different numbers of images (uneven last batch, no padding)."""
    was_training = model.training
    model.eval()
    avg = RunningAverageDict()
    n = 0
    try:
        for img, gt in batches:
            for m in evaluate_batch(model, img, gt, eval_opt, data_type):
                avg.update(m)
                n += 1
    finally:
        model.train(was_training)
    if not weight_by_count:
        return all_reduce_dict(avg.get_value(), op="mean")
    from .utils.depth_utils import METRICS
    vals = avg.get_value() if n else {k: 0.0 for k in METRICS}  # every rank reduces the same keys
    sums = {k: float(v) * n for k, v in vals.items()}
    tot = all_reduce_dict({"__count": float(n), **sums}, op="sum")
    count = tot.pop("__count")
    return {k: v / count for k, v in tot.items()}
