from .NewCRFDepth import NewCRFDepth, DispHead  # noqa: F401
