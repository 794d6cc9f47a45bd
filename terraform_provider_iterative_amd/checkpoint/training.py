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

import json
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


TORN = ("torn-risk", "signal")  # saves not taken at a step boundary


class TrainingState:
    """Checkpointer over a model + optimizer (see module docstring).

    The training loop reports each finished step with :meth:`step` (after ``opt.step()`` and
    whatever else makes up the step): that is where a preemption is saved -- on every rank at
    the same boundary -- and where periodic checkpoints are taken.  Every save records the step
    number in its metadata (``"step"``), so :meth:`resume_consistent` compares real steps.
    """

    def __init__(self, model, optimizer=None, extra: Optional[Dict[str, Any]] = None,
                 path: Optional[str] = None, device=None, **checkpointer_kwargs):
        tensors, self.host = collect(model, optimizer, extra, device)
        if not tensors:
            raise ValueError("nothing to checkpoint on the model's device")
        self.checkpointer = Checkpointer(tensors, path=path, **checkpointer_kwargs)
        self.path = path
        self.step_value: Optional[int] = None  # last step reported (or restored)

    def host_metadata(self) -> Dict[str, Any]:
        return {"host_tensors": {k: _encode(t) for k, t in self.host.items()}}

    def _metadata(self, metadata: Optional[Dict] = None) -> Dict[str, Any]:
        meta: Dict[str, Any] = {}
        if self.step_value is not None:
            meta["step"] = self.step_value
        meta.update(metadata or {})
        if isinstance(meta.get("step"), int):
            self.step_value = meta["step"]
        meta.update(self.host_metadata())
        return meta

    def step(self, step: int, metadata: Optional[Dict] = None, force: bool = False) -> bool:
        """The loop finished step ``step``: save a pending preemption here (does not return
        then), or take a periodic checkpoint when one is due (:func:`.preemption.step`).
        Returns True when a periodic checkpoint was taken."""
        self.step_value = int(step)
        return preemption.step(self.step_value, metadata, force)

    def save(self, metadata: Optional[Dict] = None):
        return self.checkpointer.save(self._metadata(metadata))

    def save_async(self, metadata: Optional[Dict] = None, codec: Optional[str] = None):
        """Periodic checkpoint that stalls the training stream only for the HBM snapshot;
        host-side tensors are captured now, with the snapshot (see
        :meth:`Checkpointer.save_async`, also for ``codec``)."""
        return self.checkpointer.save_async(self._metadata(metadata), codec=codec)

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
            if isinstance(meta.get("step"), int):
                self.step_value = meta["step"]
        return meta

    def _candidates(self, persist_path: Optional[str], key: str,
                    allow_torn: bool) -> Dict[Any, Tuple[str, Optional[int]]]:
        """``{step: (source, generation)}`` of this rank's restorable copies: the region's
        (a streamed save in flight, both slots) and the persisted file; newest copy per step."""
        out: Dict[Any, Tuple[str, Optional[int]]] = {}
        try:
            cands = self.checkpointer.candidates()
        except Exception:  # unreadable region
            cands = []
        for cand in cands:  # newest first
            meta = cand["metadata"]
            value = meta.get(key)
            if value is None or (meta.get("consistency") in TORN and not allow_torn):
                continue
            out.setdefault(value, ("region", cand["generation"]))
        if persist_path:
            import os

            from .checkpointer import describe_checkpoint

            if os.path.exists(persist_path):
                try:
                    info = describe_checkpoint(persist_path, entries=False)
                except Exception:
                    info = {}
                meta = info.get("metadata", {}) if info.get("complete") else {}
                value = meta.get(key)
                if value is not None and (meta.get("consistency") not in TORN or allow_torn):
                    out.setdefault(value, ("persist", None))
        return out

    def resume_consistent(self, persist_path: Optional[str] = None, group=None,
                          key: str = "step", allow_torn: bool = False) -> Optional[Dict]:
        """:meth:`resume` for data/tensor-parallel ranks: every rank resumes from a checkpoint
        of the same ``metadata[key]`` (the step), or none does.

        Each rank lists the steps it can restore -- a streamed save in flight, both slots of a
        ``slots=2`` region, the persisted file -- and the group (``all_gather_object``) picks
        the newest step that every rank holds.  So a rank whose last save did not complete
        (killed during the spill) makes the gang fall back to the previous common step instead
        of diverging.  Saves not taken at a step boundary (``consistency`` ``torn-risk`` /
        ``signal``: see :mod:`.preemption`) are refused unless ``allow_torn``; so are saves
        without ``metadata[key]``.  Returns None (fresh start everywhere) when no step is
        common.  Call on every rank of ``group`` (default: the world) after
        ``init_process_group``.
        """
        import torch.distributed as dist

        mine = self._candidates(persist_path, key, allow_torn)
        seen: list = [None] * dist.get_world_size(group)
        dist.all_gather_object(seen, sorted(mine, key=repr), group=group)
        common = set(seen[0] or [])
        for other in seen[1:]:
            common &= set(other or [])
        if not common:
            if any(seen):
                preemption.journal("checkpoint-disagreement", "no step common to every rank",
                                   "steps per rank %s" % json.dumps(seen)[:400])
            return None  # everybody starts fresh
        chosen = max(common)
        source, generation = mine[chosen]
        # Every rank restores that step; a rank's data may still fail verification.  Then its
        # tensors hold a partial unpack, so every rank aborts together rather than diverging.
        error: Optional[BaseException] = None
        restored = None
        try:
            if source == "region":
                restored = preemption.resume(self.checkpointer, None, generation)
            else:
                res = self.checkpointer.load(persist_path)
                preemption.journal("checkpoint-restored", persist_path,
                                   "%.1f GB/s" % res.gbps)
                restored = self.checkpointer.header().get("metadata", {})
            if restored is not None:
                self.restore_host(restored)
                self.step_value = restored.get(key) if isinstance(restored.get(key), int) \
                    else self.step_value
        except Exception as exc:  # CheckpointError, I/O errors
            error, restored = exc, None
        ok = [None] * dist.get_world_size(group)
        dist.all_gather_object(ok, error is None and restored is not None, group=group)
        if not all(ok):
            from .checkpointer import CheckpointError

            bad = [r for r, v in enumerate(ok) if not v]
            raise CheckpointError("ranks %s could not restore step %r: %s" % (
                bad, chosen, error or "restored on another rank only")) from error
        return restored

    def install(self, persist_path: Optional[str] = None) -> None:
        """Checkpoint on SIGTERM (at the next :meth:`step`; then exit 143 so the supervisor
        respawns the rank)."""
        preemption.register(self.checkpointer, persist_path)
        preemption.on_preempt(lambda: self._metadata(None))
        preemption.install()

    def close(self) -> None:
        self.checkpointer.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
