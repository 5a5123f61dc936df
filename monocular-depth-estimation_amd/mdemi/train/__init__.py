"""Restated training pieces the reference snapshot lacks (run.py, its loss,
optimizer/scheduler construction and DDP setup are missing; evidence:
output/test/wandb/latest-run/files/wandb-metadata.json:16 and the config keys
loss.*, optimizer.*, scheduler.*, train.*).  Parity for these is unpinned;
choices are documented in DESIGN.md."""
from .optim import FusedAdamW, OneCycleLR  # noqa: F401
from .loss import BinsChamferLoss, SILogLoss  # noqa: F401
from .ddp import GradAllReduce, broadcast_parameters  # noqa: F401
from .builder import Trainer, TrainLoss, build_from_config  # noqa: F401
