"""Tensor checkpoints: pack -> pinned host DRAM -> restore, with preemption handling."""
from .checkpointer import (CheckpointError, Checkpointer, DeviceEngine, TransferResult,
                           describe_checkpoint, prewarm_engine, verify_checkpoint)
from .host import HostRegion, early_prefetch, prefetch
from . import preemption
from .training import DataCursor, TrainingState, collect

__all__ = ["CheckpointError", "Checkpointer", "DeviceEngine", "TransferResult",
           "describe_checkpoint", "verify_checkpoint", "HostRegion", "TrainingState",
           "DataCursor", "collect", "preemption", "prefetch", "early_prefetch", "prewarm_engine"]
