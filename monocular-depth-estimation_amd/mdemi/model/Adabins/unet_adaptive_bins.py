"""AdaBins (mirrors model/Adabins/unet_adaptive_bins.py) on libmdemi kernels.

Public contract kept from the reference: UnetAdaptiveBins(backend, n_bins,
min_val, max_val, norm), UnetAdaptiveBins.build(n_bins, min_val, max_val),
forward(x NCHW) -> (pred (B, 1, H/2, W/2), bin_edges (B, n_bins + 1)),
get_1x_lr_params / get_10x_lr_params, state_dict keys (encoder.original_model.*,
decoder.*, adaptive_bins_layer.*, conv_out.0.*).  Inside, maps are NHWC.

The head is folded: conv_out (1x1, 128 -> n_bins) applied to the range
attention maps R = X Q^T (X the embedded map, Q the queries) equals
X (W Q)^T + b, so the logits come from one batched GEMM against the tiny
per-image matrix W Q_b and the (B, 128, H/2, W/2) range maps never reach HBM.
The bin softmax and sum_k p_k c_k run in one sweep (mdemi_binhead_nhwc)."""
import torch.nn as nn

from ... import _lib as L
from ... import functional as mf
from ..NewCRFs.uper_crf_head import bn_forward
from ..gen_efficientnet import tf_efficientnet_b5_ap, walk_features
from .miniViT import mViT


class UpSampleBN(nn.Module):
    """unet_adaptive_bins.py:8-24: bilinear (align_corners=True) to the skip size, concat,
    2 x (conv3x3 + BN + LeakyReLU)."""

    def __init__(self, skip_input, output_features):
        super().__init__()
        self._net = nn.Sequential(
            nn.Conv2d(skip_input, output_features, kernel_size=(3, 3), stride=(1, 1), padding=(1, 1)),
            nn.BatchNorm2d(output_features), nn.LeakyReLU(),
            nn.Conv2d(output_features, output_features, kernel_size=(3, 3), stride=(1, 1), padding=(1, 1)),
            nn.BatchNorm2d(output_features), nn.LeakyReLU())

    def forward(self, x, concat_with):
        f = mf.upsample_concat(x, concat_with, size=tuple(concat_with.shape[1:3]), align_corners=True)
        n = self._net
        f = bn_forward(n[1], mf.conv2d_nhwc(f, n[0].weight, n[0].bias, stride=1, pad=1), L.ACT_LEAKY)
        return bn_forward(n[4], mf.conv2d_nhwc(f, n[3].weight, n[3].bias, stride=1, pad=1), L.ACT_LEAKY)


class DecoderBN(nn.Module):
    """unet_adaptive_bins.py:27-57 (conv2 is 1x1 with padding=1, as in the reference)."""

    def __init__(self, num_features=2048, num_classes=1, bottleneck_features=2048):
        super().__init__()
        features = int(num_features)
        self.conv2 = nn.Conv2d(bottleneck_features, features, kernel_size=(1, 1), stride=(1, 1), padding=(1, 1))
        self.up1 = UpSampleBN(skip_input=features // 1 + 112 + 64, output_features=features // 2)
        self.up2 = UpSampleBN(skip_input=features // 2 + 40 + 24, output_features=features // 4)
        self.up3 = UpSampleBN(skip_input=features // 4 + 24 + 16, output_features=features // 8)
        self.up4 = UpSampleBN(skip_input=features // 8 + 16 + 8, output_features=features // 16)
        self.conv3 = nn.Conv2d(features // 16, num_classes, kernel_size=(3, 3), stride=(1, 1), padding=(1, 1))

    def forward(self, features):
        x_block0, x_block1, x_block2, x_block3, x_block4 = \
            features[4], features[5], features[6], features[8], features[11]
        x_d0 = mf.conv2d_nhwc(x_block4, self.conv2.weight, self.conv2.bias, stride=1, pad=1)
        x_d1 = self.up1(x_d0, x_block3)
        x_d2 = self.up2(x_d1, x_block2)
        x_d3 = self.up3(x_d2, x_block1)
        x_d4 = self.up4(x_d3, x_block0)
        return mf.conv2d_nhwc(x_d4, self.conv3.weight, self.conv3.bias, stride=1, pad=1)


class Encoder(nn.Module):
    """unet_adaptive_bins.py:60-73 (the walk stops at the last feature the decoder reads)."""

    def __init__(self, backend):
        super().__init__()
        self.original_model = backend

    def forward(self, x, last=11):
        return walk_features(self.original_model, x, last)


class UnetAdaptiveBins(nn.Module):
    """unet_adaptive_bins.py:76-139."""

    def __init__(self, backend, n_bins=100, min_val=0.1, max_val=10.0, norm='linear'):
        super().__init__()
        self.num_classes = n_bins
        self.min_val = min_val
        self.max_val = max_val
        self.encoder = Encoder(backend)
        self.adaptive_bins_layer = mViT(128, n_query_channels=128, patch_size=16, dim_out=n_bins,
                                        embedding_dim=128, norm=norm)
        self.decoder = DecoderBN(num_classes=128)
        self.conv_out = nn.Sequential(nn.Conv2d(128, n_bins, kernel_size=(1, 1), stride=(1, 1), padding=(0, 0)),
                                      nn.Softmax(dim=1))

    def forward(self, x, **kwargs):
        unet_out = self.decoder(self.encoder(x), **kwargs)
        queries, xe, y = self.adaptive_bins_layer.parts(unet_out)
        bin_edges, centers = mf.bins_from_raw(y, L.BINS_RELU, self.min_val, self.max_val)
        conv = self.conv_out[0]
        n_bins, nq = conv.weight.shape[:2]
        wq = mf.bgemm(conv.weight.view(n_bins, nq), queries)             # (B, n_bins, E) = W Q_b
        B, h, w, E = xe.shape
        logits = mf.bgemm(xe.view(B, h * w, E), wq, bias=conv.bias, tb=True)  # (B, HW, n_bins)
        pred = mf.bin_head_nhwc(logits.view(B, h, w, n_bins), centers)
        return pred, bin_edges

    def get_1x_lr_params(self):  # lr/10 learning rate
        return self.encoder.parameters()

    def get_10x_lr_params(self):  # lr learning rate
        for m in [self.decoder, self.adaptive_bins_layer, self.conv_out]:
            yield from m.parameters()

    def count_params(self) -> int:
        return sum(p.numel() for p in self.parameters())

    @classmethod
    def build(cls, n_bins, min_val: float, max_val: float):
        basemodel = tf_efficientnet_b5_ap(pretrained=True)
        del basemodel.bn2  # unet_adaptive_bins.py:131-134
        del basemodel.global_pool
        del basemodel.classifier
        m = cls(basemodel, n_bins=n_bins, min_val=min_val, max_val=max_val)
        print(f"Model built! #params: {m.count_params()}")
        return m
