"""Preemption-safe training state: a model's parameters/buffers + its optimizer's state.

``TrainingState(model, optimizer)`` binds every device tensor of ``model.state_dict()`` and
of the optimizer's per-parameter state into one :class:`Checkpointer` (by reference, no
copies), and carries the small host-side tensors that optimizers keep on the CPU (e.g. the
per-parameter ``step`` counters of non-capturable Adam/AdamW, which bias correction depends
on) in the checkpoint header.  ``resume()`` restores both; ``install()`` arms the SIGTERM
handler of :mod:`.preemption`.

The header also carries everything else an ordinary loop needs to continue *bit-identically*
after a respawn (``training_state``): the random number generators (torch CPU and every
initialised GPU, Python ``random``, NumPy's global generator, plus any ``generators`` handed
in), the optimizer's hyper-parameters per param group (an LR schedule changes them), the LR
scheduler, the AMP ``GradScaler``, and any object with ``state_dict``/``load_state_dict``
registered as ``stateful`` (a sampler, a data cursor: :class:`DataCursor`).  All of it is
captured at the same step boundary as the tensors.

This is the tensor-level counterpart of the reference's workdir sync: there the user script
had to re-read its own files after a spot respawn (README.md:93-101).
"""
from __future__ import annotations

import base64
import json
import random
from typing import Any, Dict, List, Optional, Tuple

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


# -- small host state as JSON (the checkpoint header) ---------------------------------------------

def to_jsonable(obj: Any) -> Any:
    """``obj`` (a ``state_dict()``-like tree) as JSON, keeping what JSON would lose: tuples,
    non-string dict keys, tensors (dtype, shape, device), NumPy arrays and bytes.  Anything
    else raises ``TypeError`` -- at construction time, not in the middle of a preemption."""
    import numpy as np

    if obj is None or isinstance(obj, (bool, int, float, str)):
        return obj
    if isinstance(obj, tuple):
        return {"__tuple__": [to_jsonable(v) for v in obj]}
    if isinstance(obj, list):
        return [to_jsonable(v) for v in obj]
    if isinstance(obj, dict):
        if all(isinstance(k, str) and not k.startswith("__") for k in obj):
            return {k: to_jsonable(v) for k, v in obj.items()}
        return {"__items__": [[to_jsonable(k), to_jsonable(v)] for k, v in obj.items()]}
    if isinstance(obj, (bytes, bytearray)):
        return {"__bytes__": base64.b64encode(bytes(obj)).decode()}
    if isinstance(obj, np.ndarray):
        return {"__ndarray__": obj.tolist(), "dtype": str(obj.dtype)}
    if isinstance(obj, np.generic):
        return obj.item()
    import torch

    if torch.is_tensor(obj):
        out = _encode(obj)
        out["__tensor__"] = True
        out["device"] = str(obj.device)
        return out
    raise TypeError("cannot carry a %s in a checkpoint header" % type(obj).__name__)


def from_jsonable(obj: Any) -> Any:
    """Inverse of :func:`to_jsonable` (tensors come back on their original device)."""
    if isinstance(obj, list):
        return [from_jsonable(v) for v in obj]
    if not isinstance(obj, dict):
        return obj
    if "__tuple__" in obj:
        return tuple(from_jsonable(v) for v in obj["__tuple__"])
    if "__items__" in obj:
        return {from_jsonable(k): from_jsonable(v) for k, v in obj["__items__"]}
    if "__bytes__" in obj:
        return base64.b64decode(obj["__bytes__"])
    if "__ndarray__" in obj:
        import numpy as np

        return np.array(obj["__ndarray__"], dtype=obj["dtype"])
    if obj.get("__tensor__"):
        import torch

        t = torch.tensor(obj["data"], dtype=getattr(torch, obj["dtype"])).reshape(obj["shape"])
        return t.to(obj.get("device", "cpu"))
    return {k: from_jsonable(v) for k, v in obj.items()}


def _b64_tensor(t) -> str:
    return base64.b64encode(t.detach().cpu().contiguous().numpy().tobytes()).decode()


def _tensor_b64(text: str):
    import numpy as np
    import torch

    return torch.from_numpy(np.frombuffer(base64.b64decode(text), dtype=np.uint8).copy())


def capture_rng() -> Dict[str, Any]:
    """Every global generator a training step may draw from: torch's CPU generator, the
    default generator of each initialised GPU, Python's ``random`` and NumPy's global one."""
    import torch

    out: Dict[str, Any] = {"torch": _b64_tensor(torch.get_rng_state()),
                           "python": to_jsonable(random.getstate())}
    try:
        import numpy as np

        out["numpy"] = to_jsonable(np.random.get_state())
    except ImportError:  # pragma: no cover
        pass
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        out["cuda"] = [_b64_tensor(torch.cuda.get_rng_state(i))
                       for i in range(torch.cuda.device_count())]
    return out


def restore_rng(state: Dict[str, Any]) -> None:
    import torch

    if "torch" in state:
        torch.set_rng_state(_tensor_b64(state["torch"]))
    if "python" in state:
        random.setstate(from_jsonable(state["python"]))
    if "numpy" in state:
        import numpy as np

        np.random.set_state(from_jsonable(state["numpy"]))
    for i, text in enumerate(state.get("cuda") or []):
        if i < torch.cuda.device_count():
            torch.cuda.set_rng_state(_tensor_b64(text), i)


class DataCursor:
    """A resumable, reproducible sample order: epoch ``e`` visits ``0..n-1`` in the
    permutation seeded by ``seed + e`` (or in order, ``shuffle=False``), and the position
    within it is part of :meth:`state_dict` -- register it as ``stateful`` and a resumed run
    draws exactly the batches the uninterrupted one would have."""

    def __init__(self, n: int, seed: int = 0, shuffle: bool = True):
        if n <= 0:
            raise ValueError("DataCursor needs at least one sample")
        self.n, self.seed, self.shuffle = int(n), int(seed), bool(shuffle)
        self.epoch = 0
        self.index = 0
        self._order: Optional[List[int]] = None

    def _permutation(self) -> List[int]:
        if self._order is None:
            if self.shuffle:
                import torch

                g = torch.Generator().manual_seed(self.seed + self.epoch)
                self._order = torch.randperm(self.n, generator=g).tolist()
            else:
                self._order = list(range(self.n))
        return self._order

    def next(self, count: int) -> List[int]:
        """The next ``count`` sample indices (crossing into the next epoch as needed)."""
        out: List[int] = []
        while len(out) < count:
            order = self._permutation()
            take = min(count - len(out), self.n - self.index)
            out.extend(order[self.index:self.index + take])
            self.index += take
            if self.index == self.n:
                self.epoch += 1
                self.index = 0
                self._order = None
        return out

    def state_dict(self) -> Dict[str, int]:
        return {"n": self.n, "seed": self.seed, "shuffle": int(self.shuffle),
                "epoch": self.epoch, "index": self.index}

    def load_state_dict(self, state: Dict[str, int]) -> None:
        if int(state["n"]) != self.n:
            raise ValueError("DataCursor over %d samples cannot resume one over %d"
                             % (self.n, int(state["n"])))
        self.seed, self.shuffle = int(state["seed"]), bool(state["shuffle"])
        self.epoch, self.index = int(state["epoch"]), int(state["index"])
        self._order = None


class TrainingState:
    """Checkpointer over a model + optimizer (see module docstring).

    The training loop reports each finished step with :meth:`step` (after ``opt.step()`` and
    whatever else makes up the step): that is where a preemption is saved -- on every rank at
    the same boundary -- and where periodic checkpoints are taken.  Every save records the step
    number in its metadata (``"step"``), so :meth:`resume_consistent` compares real steps.
    """

    def __init__(self, model, optimizer=None, extra: Optional[Dict[str, Any]] = None,
                 path: Optional[str] = None, device=None, *, lr_scheduler=None, scaler=None,
                 rng: bool = True, generators: Optional[Dict[str, Any]] = None,
                 stateful: Optional[Dict[str, Any]] = None,
                 checkpointer: Optional[Checkpointer] = None, **checkpointer_kwargs):
        tensors, self.host = collect(model, optimizer, extra, device)
        if not tensors:
            raise ValueError("nothing to checkpoint on the model's device")
        self.optimizer = optimizer
        self.lr_scheduler = lr_scheduler
        self.scaler = scaler
        self.rng = rng
        self.generators: Dict[str, Any] = dict(generators or {})
        self.stateful: Dict[str, Any] = dict(stateful or {})
        self.host_metadata()  # anything the header cannot carry fails here, not at SIGTERM
        if checkpointer is not None:  # from_materialized(): already bound to these tensors
            bound = getattr(checkpointer.plan, "_bound", [])
            if (len(bound) != len(tensors) or
                    [e.name for e in checkpointer.plan.entries] != list(tensors) or
                    any(a.data_ptr() != b.data_ptr() for a, b in zip(bound, tensors.values()))):
                raise ValueError("the checkpointer is not bound to this model's and "
                                 "optimizer's tensors")
            self.checkpointer = checkpointer
        else:
            self.checkpointer = Checkpointer(tensors, path=path, **checkpointer_kwargs)
        self.path = path if path is not None else checkpointer.path if checkpointer else None
        self.step_value: Optional[int] = None  # last step reported (or restored)

    @classmethod
    def from_materialized(cls, materialized, model, make_optimizer=None, *,
                          make_lr_scheduler=None, scaler=None, rng: bool = True,
                          generators: Optional[Dict[str, Any]] = None,
                          stateful: Optional[Dict[str, Any]] = None) -> "TrainingState":
        """Resume around the tensors of :func:`.preemption.materialize` instead of restoring
        into tensors allocated beforehand (a state too big to allocate next to its
        predecessor's; see :meth:`Checkpointer.materialize`).

        ``model`` is built without storage (``with torch.device("meta"): model = Net()``);
        its parameters and buffers become the materialized tensors
        (``load_state_dict(assign=True)``).  ``make_optimizer(model)`` then creates the
        optimizer over them, whose per-parameter state is set to the materialized tensors and
        the small host tensors of the checkpoint header (Adam's step counters);
        ``make_lr_scheduler(optimizer)`` likewise.  Everything else -- param-group
        hyper-parameters, scheduler, ``scaler``, RNGs, ``generators``, ``stateful`` objects --
        is restored as :meth:`resume` does.  The model and optimizer must be built the way the
        saving process built them (same parameter order).  Tied parameters are not re-tied.
        """
        import torch

        ck, tensors, meta = materialized
        blobs = (meta or {}).get("host_tensors", {})

        def host_tensor(name):
            blob = blobs[name]
            return torch.tensor(blob["data"], dtype=getattr(torch, blob["dtype"])).reshape(
                blob["shape"])

        module = getattr(model, "module", model)
        state = {k[len("model."):]: v for k, v in tensors.items() if k.startswith("model.")}
        for name in blobs:
            if name.startswith("model."):
                state[name[len("model."):]] = host_tensor(name)
        module.load_state_dict(state, strict=True, assign=True)
        left = [n for n, t in list(module.named_parameters()) + list(module.named_buffers())
                if t.is_meta]
        if left:  # non-persistent buffers are not in any state_dict: the caller rebuilds them
            import warnings

            warnings.warn("still on the meta device after from_materialized (not in the "
                          "checkpoint; rebuild them): %s" % ", ".join(left[:8]), stacklevel=2)
        optimizer = make_optimizer(model) if make_optimizer is not None else None
        if optimizer is not None:
            params = [p for group in optimizer.param_groups for p in group["params"]]
            for source in (tensors, blobs):
                for name in source:
                    if not name.startswith("optim."):
                        continue
                    index, key = name[len("optim."):].split(".", 1)
                    value = tensors[name] if source is tensors else host_tensor(name)
                    optimizer.state[params[int(index)]][key] = value
        extra = {k[len("extra."):]: v for k, v in tensors.items() if k.startswith("extra.")}
        lr_scheduler = make_lr_scheduler(optimizer) if make_lr_scheduler is not None else None
        out = cls(model, optimizer, extra or None, lr_scheduler=lr_scheduler, scaler=scaler,
                  rng=rng, generators=generators, stateful=stateful, checkpointer=ck)
        out.restore_host(meta or {})
        if isinstance((meta or {}).get("step"), int):
            out.step_value = meta["step"]
        return out

    def register(self, name: str, obj: Any) -> None:
        """Carry ``obj.state_dict()`` in every checkpoint and ``load_state_dict`` it on resume
        (a sampler, a data cursor, a curriculum...)."""
        if not (hasattr(obj, "state_dict") and hasattr(obj, "load_state_dict")):
            raise TypeError("%s has no state_dict()/load_state_dict()" % type(obj).__name__)
        to_jsonable(obj.state_dict())
        self.stateful[name] = obj

    def host_metadata(self) -> Dict[str, Any]:
        state: Dict[str, Any] = {}
        if self.optimizer is not None:  # lr, betas, ... (an LR schedule rewrites them)
            state["optimizer_groups"] = [to_jsonable({k: v for k, v in g.items() if k != "params"})
                                         for g in self.optimizer.param_groups]
        if self.lr_scheduler is not None:
            state["lr_scheduler"] = to_jsonable(self.lr_scheduler.state_dict())
        if self.scaler is not None:
            state["grad_scaler"] = to_jsonable(self.scaler.state_dict())
        if self.rng:
            state["rng"] = capture_rng()
        if self.generators:
            state["generators"] = {k: _b64_tensor(g.get_state())
                                   for k, g in self.generators.items()}
        if self.stateful:
            state["stateful"] = {k: to_jsonable(o.state_dict()) for k, o in self.stateful.items()}
        return {"host_tensors": {k: _encode(t) for k, t in self.host.items()},
                "training_state": state}

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
        state = metadata.get("training_state") or {}
        groups = state.get("optimizer_groups")
        if groups is not None and self.optimizer is not None:
            if len(groups) != len(self.optimizer.param_groups):
                raise ValueError("checkpoint has %d optimizer param groups, the optimizer %d"
                                 % (len(groups), len(self.optimizer.param_groups)))
            for group, saved in zip(self.optimizer.param_groups, groups):
                group.update(from_jsonable(saved))
        if "lr_scheduler" in state and self.lr_scheduler is not None:
            self.lr_scheduler.load_state_dict(from_jsonable(state["lr_scheduler"]))
        if "grad_scaler" in state and self.scaler is not None:
            self.scaler.load_state_dict(from_jsonable(state["grad_scaler"]))
        if "rng" in state and self.rng:
            restore_rng(state["rng"])
        for name, text in (state.get("generators") or {}).items():
            if name in self.generators:
                self.generators[name].set_state(_tensor_b64(text))
        for name, saved in (state.get("stateful") or {}).items():
            if name in self.stateful:
                self.stateful[name].load_state_dict(from_jsonable(saved))

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
