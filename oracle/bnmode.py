"""BatchNorm mode switch shared by the EfficientNet / AdaBins / Depthformer oracles.
TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py.

Default: training-mode BatchNorm (batch statistics), as the train step runs it.  Inside
``eval_bn()``: the running statistics, as model.eval() does (nn.BatchNorm2d in eval mode,
torch.nn.functional.batch_norm(training=False)); this is what the full-size parity tests
use for the forward, where batch statistics over a batch of 2 make the deep B5 encoder
ill-conditioned."""
import contextlib

import torch.nn.functional as F

EVAL = False


@contextlib.contextmanager
def eval_bn():
    global EVAL
    prev, EVAL = EVAL, True
    try:
        yield
    finally:
        EVAL = prev


def batch_norm(P, pre, x, eps):
    """pre: the module prefix ending in '.' (weight, bias, running_mean, running_var)."""
    if EVAL:
        # running statistics are buffers, never differentiated (a caller may hand them over as leaves)
        return F.batch_norm(x, P[pre + "running_mean"].detach(), P[pre + "running_var"].detach(), P[pre + "weight"],
                            P[pre + "bias"], training=False, eps=eps)
    return F.batch_norm(x, None, None, P[pre + "weight"], P[pre + "bias"], training=True, eps=eps)
