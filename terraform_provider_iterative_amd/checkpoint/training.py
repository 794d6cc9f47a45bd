"""Preemption-safe training state: a model's parameters/buffers + its optimizer's state.

``TrainingState(model, optimizer)`` binds every device tensor of ``model.state_dict()`` and
of the optimizer's per-parameter state into one :class:`Checkpointer` (by reference, no
copies), and carries the small host-side tensors that optimizers keep on the CPU (e.g. the
per-parameter ``step`` counters of non-capturable Adam/AdamW, which bias correction depends
on) in the checkpoint header.  ``resume()`` restores both; ``install()`` arms the SIGTERM
handler of :mod:`.preemption`.

This is the tensor-level counterpart of the reference's workdir sync: there the user script
had to re-read its own files after a spot respawn (README.md:93-101).
"""
from __future__ import annotations

from typing import Any, Dict, Optional, Tuple

from . import preemption
from .checkpointer import Checkpointer

HOST_NUMEL_LIMIT = 4096  # per host tensor carried in the JSON header


def collect(model, optimizer=None, extra: Optional[Dict[str, Any]] = None,
            device=None) -> Tuple[Dict[str, Any], Dict[str, Any]]:
    """(tensors on ``device``, small tensors elsewhere) of a model/optimizer pair.

    ``device`` defaults to the device of the model's first parameter.  Optimizer state needs
    to exist (take one step first: PyTorch creates it lazily).
    """
    import torch

    module = getattr(model, "module", model)  # DDP / FSDP-style wrappers
    state = module.state_dict(keep_vars=False)
    if device is None:
        first = next(iter(module.parameters()), None)
        device = first.device if first is not None else torch.device("cpu")
    device = torch.device(device)
    main, host = {}, {}

    def put(name, t):
        if not torch.is_tensor(t):
            return
        if t.device == device:
            main[name] = t
        else:
            if t.numel() > HOST_NUMEL_LIMIT:
                raise ValueError("%s: %d elements on %s (checkpoint device %s); move it to the "
                                 "device or checkpoint it separately" % (name, t.numel(),
                                                                        t.device, device))
            host[name] = t

    for name, t in state.items():
        put("model." + name, t)
    if optimizer is not None:
        params = [p for group in optimizer.param_groups for p in group["params"]]
        for i, param in enumerate(params):
            for key, value in optimizer.state.get(param, {}).items():
                put("optim.%d.%s" % (i, key), value)
    for name, t in (extra or {}).items():
        put("extra." + name, t)
    return main, host


def _encode(t) -> Dict[str, Any]:
    return {"dtype": str(t.dtype).replace("torch.", ""), "shape": list(t.shape),
            "data": t.detach().reshape(-1).cpu().tolist()}


def _decode_into(t, blob: Dict[str, Any]) -> None:
    import torch

    src = torch.tensor(blob["data"], dtype=getattr(torch, blob["dtype"])).reshape(blob["shape"])
    with torch.no_grad():
        t.copy_(src.to(t.device))


class TrainingState:
    """Checkpointer over a model + optimizer (see module docstring)."""

    def __init__(self, model, optimizer=None, extra: Optional[Dict[str, Any]] = None,
                 path: Optional[str] = None, device=None, **checkpointer_kwargs):
        tensors, self.host = collect(model, optimizer, extra, device)
        if not tensors:
            raise ValueError("nothing to checkpoint on the model's device")
        self.checkpointer = Checkpointer(tensors, path=path, **checkpointer_kwargs)
        self.path = path

    def host_metadata(self) -> Dict[str, Any]:
        return {"host_tensors": {k: _encode(t) for k, t in self.host.items()}}

    def save(self, metadata: Optional[Dict] = None):
        return self.checkpointer.save({**(metadata or {}), **self.host_metadata()})

    def save_async(self, metadata: Optional[Dict] = None):
        """Periodic checkpoint that stalls the training stream only for the HBM snapshot;
        host-side tensors are captured now, with the snapshot (see
        :meth:`Checkpointer.save_async`)."""
        return self.checkpointer.save_async({**(metadata or {}), **self.host_metadata()})

    def restore_host(self, metadata: Dict) -> None:
        blobs = metadata.get("host_tensors", {})
        missing = sorted(set(self.host) - set(blobs))
        if missing:
            raise ValueError("checkpoint lacks host tensors %s" % missing[:5])
        for name, t in self.host.items():
            _decode_into(t, blobs[name])

    def resume(self, persist_path: Optional[str] = None) -> Optional[Dict]:
        """Restore device tensors (host region, else ``persist_path``) and host tensors;
        returns the saved metadata or ``None`` for a fresh start."""
        meta = preemption.resume(self.checkpointer, persist_path)
        if meta is not None:
            self.restore_host(meta)
        return meta

    def resume_consistent(self, persist_path: Optional[str] = None, group=None,
                          key: str = "step") -> Optional[Dict]:
        """:meth:`resume` for data/tensor-parallel ranks: all ranks resume from checkpoints of
        the same ``metadata[key]`` or none does.  A rank whose save did not complete (killed
        during the spill) would otherwise restart from an older step than its peers; here the
        group agrees first (``all_gather_object``) and falls back to a fresh start together.
        Call on every rank of ``group`` (default: the world) after ``init_process_group``.
        """
        import torch.distributed as dist

        meta = None
        try:
            header = self.checkpointer.latest()  # complete, or streaming in (preemption)
            if header is not None:
                meta = header.get("metadata", {})
        except Exception:  # unreadable region
            meta = None
        if meta is None and persist_path:
            import os

            from .checkpointer import describe_checkpoint

            if os.path.exists(persist_path):
                try:
                    info = describe_checkpoint(persist_path, entries=False)
                    meta = info.get("metadata", {}) if info.get("complete") else None
                except Exception:
                    meta = None
        mine = None if meta is None else meta.get(key, True)
        seen = [None] * dist.get_world_size(group)
        dist.all_gather_object(seen, mine, group=group)
        if any(v is None for v in seen) or len(set(map(repr, seen))) != 1:
            return None  # disagreement: everybody starts fresh
        # The headers agree, but a rank's data may still fail verification; then its tensors
        # hold a partial unpack, so every rank aborts together rather than diverging.
        error: Optional[BaseException] = None
        try:
            restored = self.resume(persist_path)
        except Exception as exc:  # CheckpointError, I/O errors
            error, restored = exc, None
        ok = [None] * dist.get_world_size(group)
        dist.all_gather_object(ok, error is None and restored is not None, group=group)
        if not all(ok):
            from .checkpointer import CheckpointError

            bad = [r for r, v in enumerate(ok) if not v]
            raise CheckpointError("ranks %s could not restore step %r: %s" % (
                bad, mine, error or "restored on another rank only")) from error
        return restored

    def install(self, persist_path: Optional[str] = None) -> None:
        """Checkpoint on SIGTERM (then exit 143 so the supervisor respawns the rank)."""
        preemption.register(self.checkpointer, persist_path)
        preemption.on_preempt(self.host_metadata)
        preemption.install()

    def close(self) -> None:
        self.checkpointer.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
