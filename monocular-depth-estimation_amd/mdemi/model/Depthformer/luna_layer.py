"""PreNormLunaBlock / PreNormLunaLayer (mirrors model/Depthformer/luna_layer.py:134-345) on
libmdemi kernels.  hidden is token-major (B*HW, d), aux (B*K, d).

k1/v1 (both from norm(hidden)) and q2 (also from norm(hidden)) read the same
operand, so the three projections run as ONE GEMM against the stacked weights
[k1; v1; q2]; k2/v2 (both from inter_norm(out1)) likewise.  The attention
probabilities (B, heads, K, HW) / (B, heads, HW, K) are real outputs of the
reference forward, so they are materialised (softmax sweep between the QK^T
and PV GEMMs)."""
import math

import torch
import torch.nn as nn

from ... import _lib as L
from ... import functional as mf
from .feed_forward import FeedForwardBlock


class PreNormLunaBlock(nn.Module):
    def __init__(self, hidden_dim, aux_dim, qk_proj_dim, num_heads, attn_drop_prob=0.0, drop_prob=0.1):
        super().__init__()
        self.hidden_dim = hidden_dim
        self.aux_dim = aux_dim
        self.qk_proj_dim = qk_proj_dim
        self.num_heads = num_heads
        if hidden_dim % num_heads != 0:
            raise ValueError("Hidden dim not multiple of num heads.")
        self.head_dim = hidden_dim // num_heads
        self.aux_norm = nn.LayerNorm(aux_dim, eps=1e-5)
        self.inter_norm = nn.LayerNorm(aux_dim, eps=1e-5)
        self.norm = nn.LayerNorm(hidden_dim, eps=1e-5)
        self.q1_proj = nn.Linear(aux_dim, qk_proj_dim)
        self.k1_proj = nn.Linear(hidden_dim, qk_proj_dim)
        self.v1_proj = nn.Linear(hidden_dim, hidden_dim)
        self.o1_proj = nn.Linear(hidden_dim, aux_dim)
        self.q2_proj = nn.Linear(hidden_dim, qk_proj_dim)
        self.k2_proj = nn.Linear(aux_dim, qk_proj_dim)
        self.v2_proj = nn.Linear(aux_dim, hidden_dim)
        self.o2_proj = nn.Linear(hidden_dim, hidden_dim)
        self.attn_scale = math.sqrt(1.0 / self.head_dim)
        self.attn_drop = nn.Dropout(attn_drop_prob, inplace=False)
        self.drop = nn.Dropout(drop_prob, inplace=False)

    def forward(self, hidden, aux, B, HW, K):
        """hidden (B*HW, d), aux (B*K, a) -> (hidden', aux', attn1 (B,nh,K,HW), attn2 (B,nh,HW,K))."""
        d, nh, qk = self.hidden_dim, self.num_heads, self.qk_proj_dim
        tr = self.training
        # (LN(x), x) pairs: the residual paths' gradients are summed inside the LayerNorm backward
        aux_n, aux = mf.layer_norm_skip(aux, self.aux_norm.weight, self.aux_norm.bias, self.aux_norm.eps,
                                        out_b16=True)
        hidden_n, hidden = mf.layer_norm_skip(hidden, self.norm.weight, self.norm.bias, self.norm.eps, out_b16=True)
        # q/k/v projections feed the attention GEMMs: their bf16 copies from the epilogues
        q1 = mf.linear(aux_n, self.q1_proj.weight, self.q1_proj.bias, out_b16=True)         # (B*K, qk)
        w_h = torch.cat([self.k1_proj.weight, self.v1_proj.weight, self.q2_proj.weight])
        b_h = torch.cat([self.k1_proj.bias, self.v1_proj.bias, self.q2_proj.bias])
        kvq = mf.linear(hidden_n, w_h, b_h, out_b16=True)                                    # (B*HW, qk+d+qk)
        out1, attn1 = mf.attention(q1, kvq, kvq, B, K, HW, nh, qk // nh, d // nh, self.attn_scale, q_off=0,
                                   k_off=0, v_off=qk, p=self.attn_drop.p, training=tr, out_b16=True)
        out1 = mf.linear(out1, self.o1_proj.weight, self.o1_proj.bias, p=self.drop.p, training=tr)  # (B*K, a)
        aux_out = mf.add(aux, out1)
        out_n = mf.layer_norm(out1, self.inter_norm.weight, self.inter_norm.bias, self.inter_norm.eps,
                                  out_b16=True)
        w_a = torch.cat([self.k2_proj.weight, self.v2_proj.weight])
        b_a = torch.cat([self.k2_proj.bias, self.v2_proj.bias])
        kv2 = mf.linear(out_n, w_a, b_a, out_b16=True)                                       # (B*K, qk+d)
        out2, attn2 = mf.attention(kvq, kv2, kv2, B, HW, K, nh, qk // nh, d // nh, self.attn_scale,
                                   q_off=qk + d, k_off=0, v_off=qk, p=self.attn_drop.p, training=tr, out_b16=True)
        # hidden + dropout(o2_proj(out2)): the dropout and the residual add in the projection's epilogue
        out = mf.linear(out2, self.o2_proj.weight, self.o2_proj.bias, residual=hidden, p=self.drop.p, training=tr)
        return out, aux_out, attn1, attn2


class PreNormLunaLayer(nn.Module):
    """luna_layer.py:305-345: Luna + FF.  hidden NHWC (B, H, W, d) in and out."""

    def __init__(self, hidden_dim, aux_dim, qk_proj_dim, num_heads, *, feedforward_dim=None, attn_drop_prob=0.0,
                 drop_prob=0.1, act_layer=nn.GELU):
        super().__init__()
        self.luna_attn = PreNormLunaBlock(hidden_dim, aux_dim, qk_proj_dim, num_heads, attn_drop_prob, drop_prob)
        self.feed_forward = FeedForwardBlock(hidden_dim, feedforward_dim, drop_prob, act_layer, add_weight=1.0)

    def forward(self, hidden, aux):
        """hidden (B, H, W, d) NHWC, aux (B, K, a)."""
        B, h, w, d = hidden.shape
        K = aux.shape[1]
        x, a, attn1, attn2 = self.luna_attn(hidden.reshape(B * h * w, d), aux.reshape(B * K, -1), B, h * w, K)
        x = self.feed_forward(x)
        return x.view(B, h, w, d), a.view(B, K, -1), attn1, attn2
