"""mdemi — MI355X-native dense monocular-depth hot path.

Mirror of pitlover/Monocular-Depth-Estimation's model / utils surface
(``mdemi.model.{Adabins,NewCRFs,Depthformer}``, ``mdemi.utils``) running on the
hand-written gfx950 kernels of ``libmdemi.so`` (C ABI: ``include/mdemi.h``).
"""
__version__ = "0.1.0"
