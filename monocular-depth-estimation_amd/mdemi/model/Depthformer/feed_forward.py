"""FeedForwardBlock (mirrors model/Depthformer/feed_forward.py:6-46): pre-norm, fc1 -> act ->
dropout -> fc2 -> dropout, + identity; one fused Mlp op on libmdemi."""
from typing import Optional

import torch.nn as nn

from ... import functional as mf
from .layer_utils import _act_code


class FeedForwardBlock(nn.Module):
    def __init__(self, hidden_dim: int, feedforward_dim: Optional[int] = None, drop_prob: float = 0.1,
                 act_layer=nn.GELU, add_weight: float = 1.0):
        super().__init__()
        self.hidden_dim = hidden_dim
        if feedforward_dim is None:
            feedforward_dim = hidden_dim * 4
        self.feedforward_dim = feedforward_dim
        self.norm = nn.LayerNorm(hidden_dim, eps=1e-5)
        self.fc1 = nn.Linear(hidden_dim, feedforward_dim)
        self.act = act_layer()
        self.fc2 = nn.Linear(feedforward_dim, hidden_dim)
        self.drop = nn.Dropout(drop_prob, inplace=True)
        self.add_weight = add_weight
        if add_weight != 1.0:
            raise NotImplementedError("add_weight != 1 is never used by the reference")
        self._act = _act_code(act_layer)

    def forward(self, hidden):
        """hidden token-major (rows, d)."""
        # (LN(x), x): the residual path's gradient is summed inside the LayerNorm backward
        h, hidden = mf.layer_norm_skip(hidden, self.norm.weight, self.norm.bias, self.norm.eps, out_b16=True)
        return mf.mlp(h, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias, residual=hidden,
                      act=self._act, p_mid=self.drop.p, p_out=self.drop.p, training=self.training)
