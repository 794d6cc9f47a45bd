"""cty types and the msgpack/JSON value encodings Terraform uses on the plugin wire.

Types: ``"string" | "number" | "bool" | "dynamic" | ("list"|"set"|"map", T) |
("object", {name: T})``.  Unknown values are msgpack extension 0 (``d4 00 00``), exactly as
``cty/msgpack`` writes them.
"""
from __future__ import annotations

import json
from typing import Any, Dict, Tuple, Union

import msgpack

from ..models.schema import BOOL, FLOAT, INT, LIST, MAP, SET, STRING, ResourceSchema

CtyType = Union[str, Tuple[str, Any]]


class _Unknown:
    _instance = None

    def __new__(cls):
        if cls._instance is None:
            cls._instance = super().__new__(cls)
        return cls._instance

    def __repr__(self) -> str:  # pragma: no cover
        return "<unknown>"


UNKNOWN = _Unknown()
TIMEOUT_KEYS = ("create", "delete", "read", "update")


def type_json(t: CtyType) -> Any:
    if isinstance(t, str):
        return t
    kind, inner = t
    if kind == "object":
        return ["object", {k: type_json(v) for k, v in inner.items()}]
    return [kind, type_json(inner)]


def _attr_type(attr) -> CtyType:
    if attr.type in (INT, FLOAT):
        return "number"
    if attr.type == STRING:
        return "string"
    if attr.type == BOOL:
        return "bool"
    if attr.type == SET and isinstance(attr.elem, dict):
        return ("set", ("object", {k: _attr_type(a) for k, a in attr.elem.items()}))
    elem = {INT: "number", FLOAT: "number", STRING: "string", BOOL: "bool"}.get(attr.elem, "string")
    if attr.type == LIST:
        return ("list", elem)
    if attr.type == MAP:
        return ("map", elem)
    if attr.type == SET:
        return ("set", ("object", {k: _attr_type(a) for k, a in attr.elem.items()}))
    raise ValueError(attr.type)


def block_type(schema: ResourceSchema, with_timeouts: bool = True) -> CtyType:
    """cty object type of a resource as the SDK exposes it (``id`` + ``timeouts`` added)."""
    attrs: Dict[str, CtyType] = {"id": "string"}
    for name, attr in schema.attributes.items():
        attrs[name] = _attr_type(attr)
    if with_timeouts and schema.timeouts:
        attrs["timeouts"] = ("object", {k: "string" for k in TIMEOUT_KEYS
                                        if k in schema.timeouts})
    return ("object", attrs)


def _ext_hook(code: int, data: bytes):
    if code == 0:
        return UNKNOWN
    return msgpack.ExtType(code, data)


def decode_msgpack(data: bytes) -> Any:
    if not data:
        return None
    return msgpack.unpackb(data, ext_hook=_ext_hook, raw=False, strict_map_key=False)


def _conform(value: Any, t: CtyType) -> Any:
    if value is None or value is UNKNOWN:
        return value
    if t == "string":
        if isinstance(value, bool):
            return "true" if value else "false"
        return str(value) if not isinstance(value, float) or not value.is_integer() else \
            str(int(value))
    if t == "number":
        if isinstance(value, str):
            value = float(value)
        if isinstance(value, float) and value.is_integer() and abs(value) < 2 ** 63:
            return int(value)
        return value
    if t == "bool":
        return bool(value) if not isinstance(value, str) else value == "true"
    if t == "dynamic":
        return value
    kind, inner = t
    if kind in ("list", "set"):
        return [_conform(v, inner) for v in value]
    if kind == "map":
        return {str(k): _conform(v, inner) for k, v in value.items()}
    if kind == "object":
        return {k: _conform(value.get(k) if isinstance(value, dict) else None, vt)
                for k, vt in inner.items()}
    raise ValueError(t)


def _pack_default(obj):
    if obj is UNKNOWN:
        return msgpack.ExtType(0, b"\x00")
    raise TypeError("cannot encode %r" % (obj,))


def encode_msgpack(value: Any, t: CtyType) -> bytes:
    return msgpack.packb(_conform(value, t), default=_pack_default, use_bin_type=True)


def decode_json(data: bytes, t: CtyType) -> Any:
    if not data:
        return None
    return _conform(json.loads(data), t)


# ---- conversions between wire values and the resource layer's attribute dicts ---------------

def from_wire(value: Any, schema: ResourceSchema) -> Tuple[Dict[str, Any], Dict[str, float]]:
    """cty object -> (attribute dict for ``provider.resources``, timeouts in seconds).

    Unknown values become ``None``; the ``storage`` set becomes a list of dicts.
    """
    from ..models.schema import parse_duration

    attrs: Dict[str, Any] = {}
    timeouts: Dict[str, float] = {}
    for k, v in (value or {}).items():
        if k == "timeouts":
            for tk, tv in (v or {}).items():
                if isinstance(tv, str) and tv:
                    timeouts[tk] = parse_duration(tv)
            continue
        attrs[k] = None if v is UNKNOWN else _strip_unknown(v)
    for name, attr in schema.attributes.items():
        if attr.type in (INT,) and isinstance(attrs.get(name), float):
            attrs[name] = int(attrs[name])
        if attr.is_block and attrs.get(name) is None:
            attrs[name] = []
    return attrs, timeouts


def _strip_unknown(v: Any) -> Any:
    if v is UNKNOWN:
        return None
    if isinstance(v, list):
        return [_strip_unknown(x) for x in v]
    if isinstance(v, dict):
        return {k: _strip_unknown(x) for k, x in v.items()}
    return v


def to_wire(attrs: Dict[str, Any], schema: ResourceSchema,
            timeouts_value: Any = None) -> Dict[str, Any]:
    out: Dict[str, Any] = {"id": attrs.get("id") or None}
    for name, attr in schema.attributes.items():
        value = attrs.get(name)
        if attr.is_block:  # nested-block sets are never null, only empty
            value = [{k: b.get(k) for k in attr.elem} for b in (value or [])]
        out[name] = value
    if schema.timeouts:
        out["timeouts"] = timeouts_value
    return out
