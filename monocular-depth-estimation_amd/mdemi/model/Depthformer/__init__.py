"""Depthformer v8 (model/Depthformer) on libmdemi kernels."""
from .depthformer_v8 import DepthformerV8  # noqa: F401
from .decoder_v8 import DepthFormerDecoderV8  # noqa: F401
