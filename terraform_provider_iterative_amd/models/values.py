"""Task value types.

Reference: ``task/common/values.go:13-118`` (Spot, Status, Size, Event, RemoteStorage, Task,
Firewall, Environment, Variables.Enrich) and ``task/common/resource.go:8-20``.
"""
from __future__ import annotations

import datetime as _dt
import ipaddress
import os
import re
from typing import Dict, List, Mapping, Optional

from ..utils.record import field, record


class NotFoundError(Exception):
    """``common.NotFoundError`` — the backing resource does not exist."""

    def __init__(self, message: str = "resource not found"):
        super().__init__(message)


class NotImplementedError_(Exception):
    """``common.NotImplementedError`` — the backend does not implement this method.

    Named with a trailing underscore so it does not shadow the builtin; exported as
    ``NotImplementedErr`` from the package root.
    """

    def __init__(self, message: str = "resource method not implemented"):
        super().__init__(message)


NotImplementedErr = NotImplementedError_

# Spot: <0 disabled, 0 auto-priced, >0 maximum hourly price (values.go:17-22).
SPOT_DISABLED = -1.0
SPOT_ENABLED = 0.0

STATUS_RUNNING = "running"
STATUS_SUCCEEDED = "succeeded"
STATUS_FAILED = "failed"
STATUS_CODES = (STATUS_RUNNING, STATUS_SUCCEEDED, STATUS_FAILED)


def new_status() -> Dict[str, int]:
    return {code: 0 for code in STATUS_CODES}


@record
class Size:
    machine: str = "m"
    storage: int = -1


@record
class Event:
    time: _dt.datetime
    code: str
    description: List[str] = field(default_factory=list)

    def format_resource(self) -> str:
        """``resource_task.go:274-283`` event rendering."""
        return "%s: %s\n%s" % (self.time.strftime("%Y-%m-%d %H:%M:%S"), self.code,
                               "\n".join(self.description))

    def to_json(self) -> dict:
        return {"time": self.time.timestamp(), "code": self.code,
                "description": list(self.description)}

    @classmethod
    def from_json(cls, data: Mapping) -> "Event":
        return cls(time=_dt.datetime.fromtimestamp(float(data["time"]), _dt.timezone.utc),
                   code=str(data["code"]), description=list(data.get("description") or []))


@record
class RemoteStorage:
    """Pre-allocated storage container (``values.go:47-55``).

    On the node-local runtime ``container`` is an existing directory and ``path`` a
    sub-directory inside it (the k8s ``ExistingPersistentVolumeClaim`` precedent).
    """

    container: str
    path: str = ""
    config: Dict[str, str] = field(default_factory=dict)


@record
class FirewallRule:
    """``nets``/``ports`` None = allow any; empty list = allow none (``values.go:73-84``)."""

    nets: Optional[List[ipaddress.IPv4Network]] = None
    ports: Optional[List[int]] = None


@record
class Firewall:
    ingress: FirewallRule = field(default_factory=FirewallRule)
    egress: FirewallRule = field(default_factory=FirewallRule)


class Variables(dict):
    """Environment map: ``None`` values inherit from the process environment.

    Keys with a ``None`` value are treated as globs where only ``*`` is special
    (``values.go:102-118``: the reference quotes every glob metacharacter except ``*``).
    """

    def enrich(self, environ: Optional[Mapping[str, str]] = None) -> Dict[str, str]:
        environ = os.environ if environ is None else environ
        result: Dict[str, str] = {}
        for name, value in self.items():
            if value is None:
                pattern = re.compile(
                    "^" + ".*".join(re.escape(part) for part in name.split("*")) + "$", re.S)
                for key in environ:
                    if pattern.match(key):
                        result[key] = environ[key]
            else:
                result[name] = value
        return result


@record
class Environment:
    image: str = "ubuntu"
    script: str = ""
    variables: Variables = field(default_factory=Variables)
    timeout: float = 0.0  # seconds; 0 = no deadline
    directory: str = ""
    directory_out: str = ""
    exclude_list: List[str] = field(default_factory=list)


@record
class Task:
    size: Size = field(default_factory=Size)
    environment: Environment = field(default_factory=Environment)
    firewall: Firewall = field(default_factory=Firewall)
    permission_set: str = ""
    spot: float = SPOT_DISABLED
    parallelism: int = 1
    remote_storage: Optional[RemoteStorage] = None
    addresses: List[str] = field(default_factory=list)
    status: Dict[str, int] = field(default_factory=new_status)
    events: List[Event] = field(default_factory=list)

