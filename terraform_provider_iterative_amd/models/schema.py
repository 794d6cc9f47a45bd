"""Resource schemas of the provider (names, types, defaults, ForceNew, Computed, Sensitive).

Reference: ``iterative/resource_task.go:35-202`` (iterative_task),
``iterative/resource_machine.go:33-146`` (iterative_machine) and
``iterative/resource_runner.go:28-194`` (iterative_cml_runner; BASELINE.json's
"iterative_runner" is accepted as an alias).  Used by the plan/apply engine (``cli/tf.py``),
the Terraform plugin server (``provider/``) and validation.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional

from ..utils.record import field, record

STRING, INT, FLOAT, BOOL, LIST, MAP, SET = "string", "int", "float", "bool", "list", "map", "set"


@record
class Attr:
    type: str
    required: bool = False
    optional: bool = False
    computed: bool = False
    force_new: bool = False
    sensitive: bool = False
    default: Any = None
    elem: Any = STRING           # element type for list/map, or a nested schema for set blocks
    max_items: int = 0
    description: str = ""

    @property
    def is_block(self) -> bool:
        return self.type == SET and isinstance(self.elem, dict)


@record
class ResourceSchema:
    name: str
    attributes: Dict[str, Attr]
    timeouts: Dict[str, float] = field(default_factory=dict)  # seconds
    version: int = 0

    def block_attrs(self) -> Dict[str, Attr]:
        return {k: v for k, v in self.attributes.items() if v.is_block}


def _machine_attrs(startup_default: str) -> Dict[str, Attr]:
    return {
        "name": Attr(STRING, optional=True, force_new=True, default=""),
        "cloud": Attr(STRING, optional=True, force_new=True, default=""),
        "region": Attr(STRING, optional=True, force_new=True, default="us-west"),
        "image": Attr(STRING, optional=True, force_new=True, default=""),
        "spot": Attr(BOOL, optional=True, force_new=True, default=False),
        "spot_price": Attr(FLOAT, optional=True, force_new=True, default=-1.0),
        "instance_type": Attr(STRING, optional=True, force_new=True, default="m"),
        "instance_hdd_size": Attr(INT, optional=True, force_new=True, default=35),
        "instance_gpu": Attr(STRING, optional=True, force_new=True, default=""),
        "instance_ip": Attr(STRING, computed=True),
        "instance_launch_time": Attr(STRING, computed=True),
        "instance_permission_set": Attr(STRING, optional=True, force_new=True, default=""),
        "ssh_public": Attr(STRING, computed=True),
        "ssh_private": Attr(STRING, optional=True, force_new=True, default="", sensitive=True),
        "startup_script": Attr(STRING, optional=True, force_new=True, default=startup_default,
                               sensitive=True),
        "aws_security_group": Attr(STRING, optional=True, force_new=True, default=""),
        "aws_subnet_id": Attr(STRING, optional=True, force_new=True, default=""),
        "metadata": Attr(MAP, optional=True, force_new=True, elem=STRING),
    }


TASK = ResourceSchema("iterative_task", {
    "name": Attr(STRING, optional=True, force_new=True),
    "cloud": Attr(STRING, required=True, force_new=True),
    "region": Attr(STRING, optional=True, force_new=True, default="us-west"),
    "machine": Attr(STRING, optional=True, force_new=True, default="m"),
    "permission_set": Attr(STRING, optional=True, force_new=True, default=""),
    "disk_size": Attr(INT, optional=True, force_new=True, default=-1),
    "spot": Attr(FLOAT, optional=True, force_new=True, default=-1.0),
    "image": Attr(STRING, optional=True, force_new=True, default="ubuntu"),
    "ssh_public_key": Attr(STRING, computed=True, sensitive=True),
    "ssh_private_key": Attr(STRING, computed=True, sensitive=True),
    "addresses": Attr(LIST, computed=True, elem=STRING),
    "status": Attr(MAP, computed=True, elem=INT),
    "events": Attr(LIST, computed=True, elem=STRING),
    "logs": Attr(LIST, computed=True, elem=STRING),
    "script": Attr(STRING, required=True, force_new=True),
    "storage": Attr(SET, optional=True, elem={
        "workdir": Attr(STRING, optional=True, force_new=True, default=""),
        "output": Attr(STRING, optional=True, force_new=False, default=""),
        "container": Attr(STRING, optional=True, force_new=True, default=""),
        "container_opts": Attr(MAP, optional=True, force_new=True, elem=STRING),
        "exclude": Attr(LIST, optional=True, force_new=False, elem=STRING),
    }),
    "parallelism": Attr(INT, optional=True, force_new=True, default=1),
    "environment": Attr(MAP, optional=True, force_new=True, elem=STRING),
    "tags": Attr(MAP, optional=True, force_new=True, elem=STRING),
    "timeout": Attr(INT, optional=True, force_new=True, default=24 * 60 * 60),
}, timeouts={"create": 900, "read": 180, "update": 180, "delete": 900})

MACHINE = ResourceSchema("iterative_machine", _machine_attrs("#!/bin/bash"),
                         timeouts={"create": 900, "delete": 900})

_runner_attrs = {
    "repo": Attr(STRING, required=True, force_new=True),
    "token": Attr(STRING, optional=True, force_new=True, default="", sensitive=True),
    "driver": Attr(STRING, required=True, force_new=True),
    "cml_version": Attr(STRING, optional=True, force_new=True, default=""),
    "labels": Attr(STRING, optional=True, force_new=True, default="cml"),
    "idle_timeout": Attr(INT, optional=True, force_new=True, default=300),
    "single": Attr(BOOL, optional=True, force_new=True, default=False),
    "docker_volumes": Attr(LIST, optional=True, force_new=True, elem=STRING),
}
_runner_attrs.update({k: v for k, v in _machine_attrs("").items() if k not in _runner_attrs})
RUNNER = ResourceSchema("iterative_cml_runner", _runner_attrs,
                        timeouts={"create": 1200, "update": 600, "delete": 600})

SCHEMAS: Dict[str, ResourceSchema] = {
    "iterative_task": TASK,
    "iterative_machine": MACHINE,
    "iterative_cml_runner": RUNNER,
}
ALIASES = {"iterative_runner": "iterative_cml_runner"}


class SchemaError(ValueError):
    pass


def get_schema(resource_type: str) -> ResourceSchema:
    name = ALIASES.get(resource_type, resource_type)
    if name not in SCHEMAS:
        raise SchemaError("unsupported resource type %r" % resource_type)
    return SCHEMAS[name]


def _coerce(attr: Attr, value: Any, path: str) -> Any:
    if value is None:
        return None
    t = attr.type
    try:
        if t == STRING:
            if isinstance(value, bool):
                return "true" if value else "false"
            if isinstance(value, (dict, list)):
                raise TypeError
            if isinstance(value, float) and value.is_integer():
                return str(int(value))
            return str(value)
        if t == INT:
            if isinstance(value, bool):
                raise TypeError
            f = float(value)
            if not f.is_integer():
                raise TypeError
            return int(f)
        if t == FLOAT:
            if isinstance(value, bool):
                raise TypeError
            return float(value)
        if t == BOOL:
            if isinstance(value, bool):
                return value
            if value in ("true", "false"):
                return value == "true"
            raise TypeError
        if t == LIST:
            if not isinstance(value, list):
                raise TypeError
            return [_coerce(Attr(attr.elem), v, path) for v in value]
        if t == MAP:
            if not isinstance(value, dict):
                raise TypeError
            return {str(k): _coerce(Attr(attr.elem), v, path) for k, v in value.items()}
    except (TypeError, ValueError):
        raise SchemaError("%s: expected %s, got %r" % (path, t, value)) from None
    return value


def normalize(resource_type: str, config: Dict[str, Any]) -> Dict[str, Any]:
    """Validate a configuration and fill in defaults (computed attributes left ``None``).

    Nested ``storage`` blocks come in as a list of dicts (HCL block syntax).
    """
    schema = get_schema(resource_type)
    out: Dict[str, Any] = {}
    unknown = set(config) - set(schema.attributes) - {"id", "timeouts", "depends_on", "count",
                                                      "lifecycle", "provider", "for_each"}
    if unknown:
        raise SchemaError("%s: unsupported argument(s): %s" % (resource_type,
                                                             ", ".join(sorted(unknown))))
    for name, attr in schema.attributes.items():
        value = config.get(name)
        path = "%s.%s" % (resource_type, name)
        if attr.is_block:
            blocks = value or []
            if isinstance(blocks, dict):
                blocks = [blocks]
            if len(blocks) > 1:
                raise SchemaError("%s: at most one block allowed" % path)
            normalized = []
            for block in blocks:
                extra = set(block) - set(attr.elem)
                if extra:
                    raise SchemaError("%s: unsupported argument(s): %s" % (
                        path, ", ".join(sorted(extra))))
                nb = {}
                for k, a in attr.elem.items():
                    v = _coerce(a, block.get(k), "%s.%s" % (path, k))
                    nb[k] = a.default if v is None else v
                normalized.append(nb)
            out[name] = normalized
            continue
        if attr.computed and not attr.optional and not attr.required:
            out[name] = config.get(name) if name in config else None
            continue
        if value is None:
            if attr.required:
                raise SchemaError("%s: the argument %r is required" % (resource_type, name))
            value = attr.default
        out[name] = _coerce(attr, value, path)
    return out


def force_new_changes(resource_type: str, old: Dict[str, Any], new: Dict[str, Any]) -> List[str]:
    """Attributes whose change requires replacing the resource."""
    schema = get_schema(resource_type)
    changed = []
    for name, attr in schema.attributes.items():
        if attr.computed and not attr.optional and not attr.required:
            continue
        if attr.is_block:
            ob, nb = old.get(name) or [], new.get(name) or []
            if len(ob) != len(nb):
                changed.append(name)
                continue
            for o, n in zip(ob, nb):
                for k, a in attr.elem.items():
                    if a.force_new and o.get(k) != n.get(k):
                        changed.append("%s.%s" % (name, k))
            continue
        if attr.force_new and _norm(old.get(name)) != _norm(new.get(name)):
            changed.append(name)
    return changed


def in_place_changes(resource_type: str, old: Dict[str, Any], new: Dict[str, Any]) -> List[str]:
    schema = get_schema(resource_type)
    changed = []
    for name, attr in schema.attributes.items():
        if attr.is_block:
            for o, n in zip(old.get(name) or [], new.get(name) or []):
                for k, a in attr.elem.items():
                    if not a.force_new and _norm(o.get(k)) != _norm(n.get(k)):
                        changed.append("%s.%s" % (name, k))
    return changed


def _norm(value: Any) -> Any:
    if value in ({}, [], None):
        return None
    return value


def parse_duration(text: Optional[str]) -> Optional[float]:
    """Terraform timeout strings: ``"10m"``, ``"1h30m"``, ``"90s"``."""
    if not text:
        return None
    total, num = 0.0, ""
    units = {"h": 3600, "m": 60, "s": 1}
    for ch in str(text).strip():
        if ch.isdigit() or ch == ".":
            num += ch
        elif ch in units and num:
            total += float(num) * units[ch]
            num = ""
        else:
            raise SchemaError("invalid duration %r" % text)
    if num:
        total += float(num)
    return total
