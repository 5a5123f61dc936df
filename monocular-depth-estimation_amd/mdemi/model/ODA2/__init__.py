"""ODA2 ordered-swin2 (model/ODA2): the Swin encoder with replicate
padding and activation checkpointing, the ordered-reduction decoder, the wrapper."""
from .oda2_red_order_swin2 import ODA2OrderedSwin2RegModel  # noqa: F401
from .oda2_red_order_swin2_decoder import (OrderedSwin2RegDecoder, OrderedSwinBlock,  # noqa: F401
                                           OrderedSwinRegHead, PreNormOrderedSwinSA)
from .oda2_red_order_reg_decoder import PreNormDWConvFF, PreNormFF  # noqa: F401
from .oda2_swin_transformer import PatchMerging, SwinTransformer, SwinTransformerStage  # noqa: F401
