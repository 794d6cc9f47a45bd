"""Terraform state v4 (``terraform.tfstate``) for this provider's resources.

Instances are stored exactly as Terraform stores SDKv2 resources: ``attributes`` holds every
schema attribute plus ``id`` and ``timeouts``; nested blocks (``storage``) are lists of
objects; ``private`` is base64 JSON.  The local-backend lock (``.terraform.tfstate.lock.info``)
is honoured with ``flock`` so concurrent ``apply`` runs on one directory serialise, and the
previous state is kept in ``terraform.tfstate.backup``.
"""
from __future__ import annotations

import base64
import copy
import fcntl
import json
import os
from contextlib import contextmanager
from typing import Any, Dict, Iterator, List, Optional, Tuple

PROVIDER_ADDR = 'provider["registry.terraform.io/iterative/iterative"]'
TERRAFORM_VERSION = "1.5.7"
SCHEMA_TIMEOUT_KEY = "e2bfb730-ecaa-11e6-8f88-34363bc7c4c0"  # terraform-plugin-sdk timeouts key


def _uuid4() -> str:
    """Random (version 4) UUID string; avoids importing ``uuid`` (which imports ``platform``)
    on the CLI's hot path."""
    raw = bytearray(os.urandom(16))
    raw[6] = (raw[6] & 0x0F) | 0x40
    raw[8] = (raw[8] & 0x3F) | 0x80
    h = raw.hex()
    return "%s-%s-%s-%s-%s" % (h[:8], h[8:12], h[12:16], h[16:20], h[20:])


class StateError(RuntimeError):
    pass


def encode_private(timeouts: Optional[Dict[str, float]] = None) -> str:
    if not timeouts:
        return base64.b64encode(b"null").decode()
    data = {SCHEMA_TIMEOUT_KEY: {k: int(v * 1e9) for k, v in timeouts.items()}}
    return base64.b64encode(json.dumps(data).encode()).decode()


def decode_private(private: str) -> Dict[str, float]:
    try:
        data = json.loads(base64.b64decode(private or "bnVsbA==").decode())
    except ValueError:
        return {}
    if not isinstance(data, dict):
        return {}
    return {k: v / 1e9 for k, v in (data.get(SCHEMA_TIMEOUT_KEY) or {}).items()}


def address(type_: str, name: str, index: Any = None) -> str:
    if index is None:
        return "%s.%s" % (type_, name)
    return "%s.%s[%s]" % (type_, name, json.dumps(index))


def parse_address(addr: str) -> Tuple[str, str, Any]:
    index = None
    if addr.endswith("]") and "[" in addr:
        addr, _, raw = addr[:-1].partition("[")
        index = json.loads(raw)
    type_, _, name = addr.partition(".")
    if not type_ or not name:
        raise StateError("invalid resource address %r" % addr)
    return type_, name, index


class State:
    def __init__(self, data: Optional[Dict[str, Any]] = None):
        self.data = data or {"version": 4, "terraform_version": TERRAFORM_VERSION, "serial": 0,
                             "lineage": _uuid4(), "outputs": {}, "resources": [],
                             "check_results": None}
        if self.data.get("version") != 4:
            raise StateError("unsupported state version %r" % self.data.get("version"))

    # -- persistence ------------------------------------------------------------------------------
    @classmethod
    def load(cls, path: str) -> "State":
        if not os.path.exists(path) or os.path.getsize(path) == 0:
            return cls()
        with open(path) as handle:
            return cls(json.load(handle))

    def save(self, path: str) -> None:
        self.data["serial"] = int(self.data.get("serial", 0)) + 1
        if os.path.exists(path):
            with open(path) as src, open(path + ".backup", "w") as dst:
                dst.write(src.read())
        tmp = path + ".tmp"
        with open(tmp, "w") as handle:
            json.dump(self.data, handle, indent=2)
            handle.write("\n")
        os.replace(tmp, path)

    @staticmethod
    @contextmanager
    def locked(path: str, operation: str = "OperationTypeApply") -> Iterator[None]:
        lock_path = os.path.join(os.path.dirname(os.path.abspath(path)),
                                 ".terraform.tfstate.lock.info")
        fd = os.open(lock_path, os.O_RDWR | os.O_CREAT, 0o644)
        try:
            try:
                fcntl.flock(fd, fcntl.LOCK_EX | fcntl.LOCK_NB)
            except BlockingIOError:
                raise StateError("Error acquiring the state lock (%s is held by another "
                                 "process)" % lock_path) from None
            info = {"ID": _uuid4(), "Operation": operation, "Info": "",
                    "Who": "%s@%s" % (os.environ.get("USER", "?"), os.uname().nodename),
                    "Version": TERRAFORM_VERSION, "Path": os.path.abspath(path)}
            os.ftruncate(fd, 0)
            os.write(fd, json.dumps(info).encode())
            yield
        finally:
            try:
                os.ftruncate(fd, 0)
                fcntl.flock(fd, fcntl.LOCK_UN)
            finally:
                os.close(fd)
                try:
                    os.unlink(lock_path)
                except FileNotFoundError:
                    pass

    # -- resources --------------------------------------------------------------------------------
    def _resource(self, type_: str, name: str, create: bool = False) -> Optional[Dict[str, Any]]:
        for res in self.data["resources"]:
            if res.get("mode") == "managed" and res["type"] == type_ and res["name"] == name:
                return res
        if not create:
            return None
        res = {"mode": "managed", "type": type_, "name": name, "provider": PROVIDER_ADDR,
               "instances": []}
        self.data["resources"].append(res)
        return res

    def instances(self) -> List[Tuple[str, str, Any, Dict[str, Any]]]:
        out = []
        for res in self.data["resources"]:
            if res.get("mode") != "managed":
                continue
            for inst in res.get("instances", []):
                out.append((res["type"], res["name"], inst.get("index_key"), inst))
        return out

    def get(self, type_: str, name: str, index: Any = None) -> Optional[Dict[str, Any]]:
        res = self._resource(type_, name)
        if not res:
            return None
        for inst in res["instances"]:
            if inst.get("index_key") == index:
                return inst
        return None

    def put(self, type_: str, name: str, attributes: Dict[str, Any], index: Any = None,
            timeouts: Optional[Dict[str, float]] = None, sensitive: Optional[List[str]] = None,
            schema_version: int = 0) -> Dict[str, Any]:
        res = self._resource(type_, name, create=True)
        attrs = copy.deepcopy(attributes)
        attrs.setdefault("timeouts", None)
        inst = {"schema_version": schema_version, "attributes": attrs,
                "sensitive_attributes": [[{"type": "get_attr", "value": s}] for s in sensitive or []],
                "private": encode_private(timeouts)}
        if index is not None:
            inst["index_key"] = index
        for i, old in enumerate(res["instances"]):
            if old.get("index_key") == index:
                res["instances"][i] = inst
                break
        else:
            res["instances"].append(inst)
        return inst

    def remove(self, type_: str, name: str, index: Any = None) -> bool:
        res = self._resource(type_, name)
        if not res:
            return False
        before = len(res["instances"])
        res["instances"] = [i for i in res["instances"] if i.get("index_key") != index]
        if not res["instances"]:
            self.data["resources"].remove(res)
        return len(res.get("instances", [])) != before or before > 0

    def addresses(self) -> List[str]:
        return [address(t, n, i) for t, n, i, _ in self.instances()]

    def attribute_tree(self) -> Dict[str, Dict[str, Any]]:
        """``{type: {name: attrs | [attrs...]}}`` for evaluating outputs."""
        tree: Dict[str, Dict[str, Any]] = {}
        for type_, name, index, inst in self.instances():
            bucket = tree.setdefault(type_, {})
            if index is None:
                bucket[name] = inst["attributes"]
            else:
                bucket.setdefault(name, [])
                bucket[name].append(inst["attributes"])
        return tree
