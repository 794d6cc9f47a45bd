"""Tensor flatten ("pack") into one CRC-tiled stream and its inverse ("unpack").

Stream layout: tensor payloads in plan order, each starting at a multiple of
:data:`SEG_ALIGN` bytes, gaps zero-filled; tile ``t`` covers bytes ``[t*tile, (t+1)*tile)``
and carries the standard CRC32C of those bytes.  Non-contiguous tensors (<= 6 dims) are
moved straight from/to their storage, no temporary contiguous copy: the view is first
canonicalised (size-1 dims dropped, mergeable dims merged) and classified for the kernels
(``csrc/hip/kernels.hip``): sliced rows move as 16-byte vectors, transposed matrices through
LDS-tiled transposes, anything else element by element.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Mapping, Sequence, Tuple, Union

import numpy as np

from ._loader import hip, native
from .hashing import DEFAULT_TILE_BYTES, _is_device_tensor, _stream

SEG_ALIGN = 256
MAX_DIMS = 6
SEG_CONTIG, SEG_STRIDED, SEG_ROWS, SEG_TRANSPOSE = 0, 1, 2, 3  # csrc/hip/tpi_hip.h
SEG_DTYPE = np.dtype([
    ("ptr", "<u8"), ("off", "<u8"), ("nbytes", "<u8"), ("kind", "<u4"), ("elem", "<u4"),
    ("ndim", "<i4"), ("pad", "<i4"), ("sizes", "<i8", (MAX_DIMS,)),
    ("strides", "<i8", (MAX_DIMS,)),
])
assert SEG_DTYPE.itemsize == 136


def align_up(value: int, alignment: int = SEG_ALIGN) -> int:
    return (value + alignment - 1) // alignment * alignment


def canonical_view(shape, stride) -> List[Tuple[int, int]]:
    """(size, stride) dims of a view with size-1 dims dropped and mergeable dims merged
    (outer dim d folds into inner dim d+1 when stride[d] == stride[d+1] * size[d+1])."""
    merged: List[Tuple[int, int]] = []
    for size, st in zip(shape, stride):
        size, st = int(size), int(st)
        if size == 1:
            continue
        if merged and merged[-1][1] == st * size:
            merged[-1] = (merged[-1][0] * size, st)
        else:
            merged.append((size, st))
    return merged or [(1, 1)]


def classify_view(dims: List[Tuple[int, int]], elem: int) -> int:
    """Kernel path for a canonical view (see ``tpi_hip.h``)."""
    strides = [st for _, st in dims]
    if len(dims) == 1 and strides[0] == 1:
        return SEG_CONTIG
    if any(st <= 0 for st in strides):  # expanded (stride 0) views: element path
        return SEG_STRIDED
    if strides[-1] == 1:
        return SEG_ROWS
    if elem in (1, 2, 4, 8) and ((len(dims) == 2 and strides[0] == 1) or
                                 (len(dims) == 3 and strides[1] == 1)):
        return SEG_TRANSPOSE
    return SEG_STRIDED


@dataclass
class TensorEntry:
    name: str
    dtype: str
    shape: Tuple[int, ...]
    nbytes: int
    offset: int

    def to_json(self) -> dict:
        return {"name": self.name, "dtype": self.dtype, "shape": list(self.shape),
                "nbytes": self.nbytes, "offset": self.offset}

    @classmethod
    def from_json(cls, data: Mapping) -> "TensorEntry":
        return cls(name=data["name"], dtype=data["dtype"], shape=tuple(data["shape"]),
                   nbytes=int(data["nbytes"]), offset=int(data["offset"]))


def _dtype_name(t) -> str:
    return str(t.dtype).replace("torch.", "")


TensorsLike = Union[Mapping[str, "object"], Sequence["object"]]


def _named(tensors: TensorsLike) -> List[Tuple[str, "object"]]:
    if isinstance(tensors, Mapping):
        return list(tensors.items())
    return [(str(i), t) for i, t in enumerate(tensors)]


class PackPlan:
    """Layout of a set of tensors in the packed stream plus their segment descriptors."""

    def __init__(self, entries: List[TensorEntry], total: int, tile_bytes: int):
        self.entries = entries
        self.total = total
        self.tile_bytes = tile_bytes
        self.segs = np.zeros(len(entries), dtype=SEG_DTYPE)
        self.device = None
        self._dev_segs = None

    @property
    def ntiles(self) -> int:
        return (self.total + self.tile_bytes - 1) // self.tile_bytes

    @classmethod
    def from_tensors(cls, tensors: TensorsLike, tile_bytes: int = DEFAULT_TILE_BYTES) -> "PackPlan":
        if tile_bytes <= 0 or tile_bytes % 4096:
            raise ValueError("tile_bytes must be a positive multiple of 4096")
        named = _named(tensors)
        if not named:
            raise ValueError("nothing to pack")
        entries, off = [], 0
        for name, t in named:
            nbytes = t.numel() * t.element_size()
            entries.append(TensorEntry(name, _dtype_name(t), tuple(t.shape), nbytes, off))
            off = align_up(off + nbytes)
        plan = cls(entries, max(off, SEG_ALIGN), tile_bytes)
        plan.bind(tensors)
        return plan

    @classmethod
    def from_entries(cls, entries: List[TensorEntry], total: int, tile_bytes: int) -> "PackPlan":
        return cls(list(entries), total, tile_bytes)

    def bind(self, tensors: TensorsLike) -> "PackPlan":
        """(Re)point the segment descriptors at ``tensors`` (same names/shapes/dtypes)."""
        named = _named(tensors)
        if len(named) != len(self.entries):
            raise ValueError("tensor count does not match the plan")
        devices = set()
        for i, ((name, t), e) in enumerate(zip(named, self.entries)):
            if name != e.name or tuple(t.shape) != e.shape or _dtype_name(t) != e.dtype:
                raise ValueError("tensor %r does not match plan entry %r" % (name, e.name))
            devices.add(str(t.device))
            s = self.segs[i]
            s["ptr"] = t.data_ptr()
            s["off"] = e.offset
            s["nbytes"] = e.nbytes
            s["elem"] = t.element_size()
            dims = [(1, 1)] if t.is_contiguous() or t.numel() <= 1 else \
                canonical_view(t.shape, t.stride())
            kind = classify_view(dims, t.element_size())
            if kind == SEG_CONTIG:
                s["kind"], s["ndim"] = SEG_CONTIG, 0
            else:
                if len(dims) > MAX_DIMS:
                    raise ValueError("non-contiguous tensors with more than %d (merged) dims "
                                     "are not supported (%r)" % (MAX_DIMS, name))
                s["kind"], s["ndim"] = kind, len(dims)
                s["sizes"][:] = 1
                s["strides"][:] = 0
                s["sizes"][:len(dims)] = [d[0] for d in dims]
                s["strides"][:len(dims)] = [d[1] for d in dims]
        if len(devices) != 1:
            raise ValueError("all tensors of a plan must live on one device, got %s" % devices)
        self.device = devices.pop()
        self._dev_segs = None
        self._bound = [t for _, t in named]  # descriptors hold raw pointers: keep them alive
        return self

    def unbind(self) -> None:
        """Drop the bound tensors (their memory may go once the caller's references do); the
        descriptors' pointers are cleared with them."""
        self._bound = []
        self._dev_segs = None
        self.segs["ptr"] = 0

    @property
    def on_device(self) -> bool:
        return self.device is not None and self.device.startswith("cuda")

    def device_segments(self):
        """The descriptor array as a device uint8 tensor (uploaded once per bind)."""
        import torch

        if self._dev_segs is None:
            host = torch.from_numpy(self.segs.view(np.uint8).copy())
            self._dev_segs = host.to(self.device)
        return self._dev_segs

    def header(self) -> Dict:
        return {"tile_bytes": self.tile_bytes, "total": self.total,
                "entries": [e.to_json() for e in self.entries]}


def pack(plan: PackPlan, out=None, threads: int = 8):
    """Pack the bound tensors into ``out`` (device uint8 tensor / host buffer of
    ``plan.total`` bytes).  Returns ``(out, crcs)``."""
    if plan.on_device:
        import torch

        dev = torch.device(plan.device)
        if out is None:
            out = torch.empty(plan.total, dtype=torch.uint8, device=dev)
        crcs = torch.empty(plan.ntiles, dtype=torch.int32, device=dev)
        segs = plan.device_segments()
        lib = hip()
        with torch.cuda.device(dev):
            lib.check(lib.tpi_pack_device(segs.data_ptr(), plan.segs.ctypes.data,
                                          len(plan.entries), plan.total, out.data_ptr(),
                                          plan.tile_bytes, crcs.data_ptr(), _stream(out)),
                      "pack")
        return out, crcs
    if out is None:
        out = np.empty(plan.total, dtype=np.uint8)
    from .hashing import host_buffer

    addr, nbytes, _keep = host_buffer(out)
    if nbytes < plan.total:
        raise ValueError("output buffer too small")
    crcs = np.zeros(plan.ntiles, dtype=np.uint32)
    native().pack_ptr(plan.segs, plan.total, addr, plan.tile_bytes, crcs.ctypes.data, threads)
    return out, crcs


def unpack(plan: PackPlan, stream, crcs, threads: int = 8) -> Tuple[int, int]:
    """Verify every tile of ``stream`` against ``crcs`` and scatter into the bound tensors.

    Returns ``(bad_tiles, first_bad_tile)`` (``(0, -1)`` when everything verified).  Tiles
    are scattered even when they fail verification so callers can decide what to do.
    """
    if plan.on_device:
        import torch

        dev = torch.device(plan.device)
        if not _is_device_tensor(stream):
            raise TypeError("device plan needs a device stream buffer")
        crc_t = crcs if _is_device_tensor(crcs) else torch.as_tensor(
            np.asarray(crcs, dtype=np.uint32).view(np.int32)).to(dev)
        bad = torch.tensor([0, -1], dtype=torch.int64, device=dev)
        segs = plan.device_segments()
        lib = hip()
        with torch.cuda.device(dev):
            lib.check(lib.tpi_unpack_device(segs.data_ptr(), plan.segs.ctypes.data,
                                            len(plan.entries), plan.total, stream.data_ptr(),
                                            plan.tile_bytes, crc_t.data_ptr(), bad.data_ptr(),
                                            _stream(stream)), "unpack")
        count, first = (int(v) for v in bad.cpu().tolist())
        return count, (first if count else -1)
    from .hashing import host_buffer

    addr, nbytes, _keep = host_buffer(stream)
    crc_arr = np.ascontiguousarray(np.asarray(crcs).view(np.uint32)
                                   if np.asarray(crcs).dtype != np.uint32 else crcs)
    bad, first = native().unpack_ptr(plan.segs, plan.total, addr, plan.tile_bytes,
                                     crc_arr.ctypes.data, threads)
    return int(bad), int(first)


def crc_array(crcs) -> np.ndarray:
    """Host ``np.uint32`` view of a CRC result (device int32 tensor or numpy)."""
    if hasattr(crcs, "cpu"):
        return crcs.cpu().numpy().view(np.uint32)
    return np.asarray(crcs).view(np.uint32) if np.asarray(crcs).dtype != np.uint32 else np.asarray(crcs)

