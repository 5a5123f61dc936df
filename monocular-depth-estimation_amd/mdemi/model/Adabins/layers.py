"""mViT building blocks (mirrors model/Adabins/layers.py) on libmdemi kernels, NHWC inside.

PatchTransformerEncoder keeps the reference's parameters (embedding_encoder,
positional_encodings, an nn.TransformerEncoder(128, 4 heads, ff 1024) used as a
parameter container) and runs the post-norm encoder layers as fused GEMMs +
the batched-attention op, with the layers' dropout (p = 0.1) applied in
training exactly where nn.TransformerEncoderLayer applies it."""
import torch
import torch.nn as nn

from ... import _lib as L
from ... import functional as mf


def transformer_encoder_layer(layer: nn.TransformerEncoderLayer, t, B, S, training):
    """nn.TransformerEncoderLayer (post-norm, ReLU) on token-major t [B*S, E]."""
    sa = layer.self_attn
    E = t.shape[-1]
    heads = sa.num_heads
    hd = E // heads
    qkv = mf.linear(t, sa.in_proj_weight, sa.in_proj_bias)
    o, _ = mf.attention(qkv, qkv, qkv, B, S, S, heads, hd, hd, hd ** -0.5, q_off=0, k_off=E, v_off=2 * E,
                        p=sa.dropout, training=training)
    # t + dropout1(out_proj(o)): dropout and residual add in the projection's epilogue
    x = mf.linear(o, sa.out_proj.weight, sa.out_proj.bias, residual=t, p=layer.dropout1.p, training=training)
    x = mf.layer_norm(x, layer.norm1.weight, layer.norm1.bias, layer.norm1.eps)
    y = mf.mlp(x, layer.linear1.weight, layer.linear1.bias, layer.linear2.weight, layer.linear2.bias, residual=x,
               act=L.ACT_RELU, p_mid=layer.dropout.p, p_out=layer.dropout2.p, training=training)
    return mf.layer_norm(y, layer.norm2.weight, layer.norm2.bias, layer.norm2.eps)


class PatchTransformerEncoder(nn.Module):
    """layers.py:5-31.  forward(x NHWC) -> tokens (B, S, E) (the reference's (S, N, E), batch-major)."""

    def __init__(self, in_channels, patch_size=10, embedding_dim=128, num_heads=4):
        super().__init__()
        encoder_layers = nn.TransformerEncoderLayer(embedding_dim, num_heads, dim_feedforward=1024)
        self.transformer_encoder = nn.TransformerEncoder(encoder_layers, num_layers=4, enable_nested_tensor=False)
        self.embedding_encoder = nn.Conv2d(in_channels, embedding_dim, kernel_size=(patch_size, patch_size),
                                           stride=(patch_size, patch_size), padding=(0, 0))
        self.positional_encodings = nn.Parameter(torch.rand(500, embedding_dim), requires_grad=True)

    def forward(self, x):
        p = self.embedding_encoder.kernel_size[0]
        emb = mf.conv2d_nhwc(x, self.embedding_encoder.weight, self.embedding_encoder.bias, stride=p, pad=0)
        B, h, w, E = emb.shape
        S = h * w
        if S > self.positional_encodings.shape[0]:
            raise ValueError(f"{S} patches exceed the {self.positional_encodings.shape[0]} positional encodings")
        t = mf.add_rows_broadcast(emb.view(B, S, E), self.positional_encodings).view(B * S, E)
        for layer in self.transformer_encoder.layers:
            t = transformer_encoder_layer(layer, t, B, S, self.training)
        return t.view(B, S, E)


class PixelWiseDotProduct(nn.Module):
    """layers.py:34-43: x (B, H, W, C) NHWC . K (B, cout, C) -> (B, H, W, cout)."""

    def forward(self, x, K):
        n, h, w, c = x.shape
        _, cout, ck = K.shape
        assert c == ck, "Number of channels in x and Embedding dimension (at dim 2) of K matrix must match"
        return mf.bgemm(x.reshape(n, h * w, c), K, tb=True).view(n, h, w, cout)
