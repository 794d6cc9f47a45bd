"""Small helpers (reference: ``iterative/utils/helpers.go``)."""
from __future__ import annotations

import os
import re
from typing import Iterable, Optional

_SEMVER = re.compile(r"^v?(\d+)\.(\d+)\.(\d+)(?:[-+].*)?$")


def get_cml(version: str = "") -> str:
    """Shell snippet installing CML (``GetCML``).  Without network access the node runtime
    expects ``cml`` on PATH; the snippet is still rendered for remote images."""
    if not version:
        return "command -v cml >/dev/null 2>&1 || sudo npm install --global @dvcorg/cml"
    match = _SEMVER.match(version)
    if match:
        return "command -v cml >/dev/null 2>&1 || sudo npm install --global @dvcorg/cml@v%s" % \
            ".".join(match.groups())
    return "command -v cml >/dev/null 2>&1 || sudo npm install --global %s" % version


def machine_prefix(data: dict) -> str:
    return "machine.0." if data.get("machine") else ""


def multi_env_load_first(names: Iterable[str], environ=None) -> str:
    environ = os.environ if environ is None else environ
    for name in names:
        value = environ.get(name)
        if value:
            return value
    return ""


def set_id(data: dict, new_id: Optional[str] = None) -> str:
    """Assign a ``cml-`` identifier when the resource has none (``SetId``)."""
    if not data.get("id"):
        from .identifier import new_random_identifier

        data["id"] = new_id or new_random_identifier(data.get("name") or "").long().replace(
            "tpi-", "cml-", 1)
    return data["id"]
