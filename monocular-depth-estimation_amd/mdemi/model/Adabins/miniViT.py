"""mViT (mirrors model/Adabins/miniViT.py) on libmdemi kernels, NHWC inside."""
import torch.nn as nn

from ... import _lib as L
from ... import functional as mf
from .layers import PatchTransformerEncoder, PixelWiseDotProduct


class mViT(nn.Module):
    """miniViT.py:7-48.  forward(x NHWC) -> (bin_widths_normed (B, dim_out), range_attention_maps NHWC)."""

    def __init__(self, in_channels, n_query_channels=128, patch_size=16, dim_out=256, embedding_dim=128,
                 num_heads=4, norm='linear'):
        super().__init__()
        self.norm = norm
        self.n_query_channels = n_query_channels
        self.patch_transformer = PatchTransformerEncoder(in_channels, patch_size, embedding_dim, num_heads)
        self.dot_product_layer = PixelWiseDotProduct()
        self.embedding_conv = nn.Conv2d(in_channels, embedding_dim, kernel_size=3, stride=1, padding=1)
        self.regressor = nn.Sequential(nn.Linear(embedding_dim, 256), nn.LeakyReLU(), nn.Linear(256, 256),
                                       nn.LeakyReLU(), nn.Linear(256, dim_out))

    def parts(self, x):
        """-> (queries (B, nq, E), embedded map NHWC (B, H, W, E), regressor output (B, dim_out))."""
        if self.norm != "linear":
            raise NotImplementedError("mViT: only norm='linear' (the reference default) runs on libmdemi")
        tgt = self.patch_transformer(x)
        xe = mf.conv2d_nhwc(x, self.embedding_conv.weight, self.embedding_conv.bias, stride=1, pad=1)
        head = mf.take_rows(tgt, 0, 1).view(tgt.shape[0], -1)
        queries = mf.take_rows(tgt, 1, self.n_query_channels)
        r = self.regressor
        y = mf.linear_act(head, r[0].weight, r[0].bias, L.ACT_LEAKY)
        y = mf.linear_act(y, r[2].weight, r[2].bias, L.ACT_LEAKY)
        y = mf.linear(y, r[4].weight, r[4].bias)
        return queries, xe, y

    def forward(self, x):
        queries, xe, y = self.parts(x)
        range_attention_maps = self.dot_product_layer(xe, queries)
        widths, _, _ = mf.bins_from_raw(y, L.BINS_RELU, 0.0, 1.0, with_widths=True)  # relu(y)+0.1, normalised
        return widths, range_attention_maps
