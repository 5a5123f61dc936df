"""AdaBins (model/Adabins) on libmdemi kernels."""
from .miniViT import mViT  # noqa: F401
from .unet_adaptive_bins import UnetAdaptiveBins  # noqa: F401
