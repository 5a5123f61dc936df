"""SelfAttentionBlock / ViTLayer (mirrors model/Depthformer/self_attention.py:7-88 and
vit_layer.py:9-44) on libmdemi kernels; q/k/v projections as one stacked GEMM."""
import math
from typing import Optional

import torch
import torch.nn as nn

from ... import functional as mf
from .feed_forward import FeedForwardBlock


class SelfAttentionBlock(nn.Module):
    def __init__(self, hidden_dim, key_query_dim, num_heads, attn_drop_prob=0.0, drop_prob=0.1):
        super().__init__()
        self.hidden_dim = hidden_dim
        self.key_query_dim = key_query_dim
        self.num_heads = num_heads
        if (hidden_dim % num_heads != 0) or (key_query_dim % num_heads != 0):
            raise ValueError("Hidden dim not multiple of num heads.")
        self.head_dim = key_query_dim // num_heads
        self.norm = nn.LayerNorm(hidden_dim, eps=1e-5)
        self.query_proj = nn.Linear(hidden_dim, key_query_dim)
        self.key_proj = nn.Linear(hidden_dim, key_query_dim)
        self.value_proj = nn.Linear(hidden_dim, hidden_dim)
        self.out_proj = nn.Linear(hidden_dim, hidden_dim)
        self.attn_scale = math.sqrt(1.0 / self.head_dim)
        self.attn_drop = nn.Dropout(attn_drop_prob, inplace=False)
        self.drop = nn.Dropout(drop_prob, inplace=True)

    def forward(self, hidden, B, S):
        """hidden (B*S, d) -> (hidden', attn (B, nh, S, S))."""
        kq, d, nh = self.key_query_dim, self.hidden_dim, self.num_heads
        h, hidden = mf.layer_norm_skip(hidden, self.norm.weight, self.norm.bias, self.norm.eps, out_b16=True)
        w = torch.cat([self.query_proj.weight, self.key_proj.weight, self.value_proj.weight])
        b = torch.cat([self.query_proj.bias, self.key_proj.bias, self.value_proj.bias])
        qkv = mf.linear(h, w, b, out_b16=True)  # the attention GEMMs' operand: bf16 copy from the epilogue
        o, attn = mf.attention(qkv, qkv, qkv, B, S, S, nh, kq // nh, d // nh, self.attn_scale, q_off=0, k_off=kq,
                               v_off=2 * kq, p=self.attn_drop.p, training=self.training, out_b16=True)
        # hidden + dropout(out_proj(o)): dropout and residual add in the projection's epilogue
        out = mf.linear(o, self.out_proj.weight, self.out_proj.bias, residual=hidden, p=self.drop.p,
                        training=self.training)
        return out, attn


class ViTLayer(nn.Module):
    def __init__(self, hidden_dim, key_query_dim, num_heads, *, num_repeat=1, feedforward_dim: Optional[int] = None,
                 attn_drop_prob=0.0, drop_prob=0.1, act_layer=nn.GELU):
        super().__init__()
        if num_repeat < 1:
            raise ValueError("num_repeat is less than 1.")
        self.num_repeat = num_repeat
        self.self_attn = SelfAttentionBlock(hidden_dim, key_query_dim, num_heads, attn_drop_prob, drop_prob)
        self.feed_forward = FeedForwardBlock(hidden_dim, feedforward_dim, drop_prob, act_layer)

    def forward(self, hidden):
        """hidden (B, S, d) -> ((B, S, d), attn)."""
        B, S, d = hidden.shape
        x = hidden.reshape(B * S, d)
        attn = None
        for _ in range(self.num_repeat):
            x, attn = self.self_attn(x, B, S)
            x = self.feed_forward(x)
        return x.view(B, S, d), attn
