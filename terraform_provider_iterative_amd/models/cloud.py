"""Cloud descriptor.

Reference: ``task/common/cloud.go:8-69``.  The reference's providers are remote clouds
(``aws``/``gcp``/``az``/``k8s``); this framework adds the two node-local providers that
actually run work here: ``local`` (CPU processes) and ``mi355x`` (1-8 GPUs of this node).
The remote providers are kept as recognised names so configurations parse and fail with a
clear diagnostic instead of an "unknown provider" error (see ``backends/remote.py``).
"""
from __future__ import annotations

import os
from typing import Dict, Mapping, Optional

from ..utils.record import field, record

PROVIDER_AWS = "aws"
PROVIDER_GCP = "gcp"
PROVIDER_AZ = "az"
PROVIDER_K8S = "k8s"
PROVIDER_LOCAL = "local"
PROVIDER_MI355X = "mi355x"

REMOTE_PROVIDERS = (PROVIDER_AWS, PROVIDER_GCP, PROVIDER_AZ, PROVIDER_K8S)
NODE_PROVIDERS = (PROVIDER_LOCAL, PROVIDER_MI355X)
ALL_PROVIDERS = NODE_PROVIDERS + REMOTE_PROVIDERS

# Default resource timeouts (resource_task.go:197-202, cmd/leo/root.go:34-39), seconds.
DEFAULT_TIMEOUTS = {"create": 15 * 60.0, "read": 3 * 60.0, "update": 3 * 60.0,
                    "delete": 15 * 60.0}


@record
class Timeouts:
    create: float = DEFAULT_TIMEOUTS["create"]
    read: float = DEFAULT_TIMEOUTS["read"]
    update: float = DEFAULT_TIMEOUTS["update"]
    delete: float = DEFAULT_TIMEOUTS["delete"]


@record
class AWSCredentials:
    access_key_id: str = ""
    secret_access_key: str = ""
    session_token: str = ""


@record
class GCPCredentials:
    application_credentials: str = ""


@record
class AZCredentials:
    client_id: str = ""
    client_secret: str = ""
    subscription_id: str = ""
    tenant_id: str = ""


@record
class K8SCredentials:
    config: str = ""


@record
class NodeCredentials:
    """Credentials of the node-local runtime: where task state lives.

    ``state_root`` plays the role of the cloud account: every task of this provider keeps
    its storage (``data/``, ``reports/``) and supervisor state below it.
    """

    state_root: str = ""


@record
class Credentials:
    aws: Optional[AWSCredentials] = None
    gcp: Optional[GCPCredentials] = None
    az: Optional[AZCredentials] = None
    k8s: Optional[K8SCredentials] = None
    node: Optional[NodeCredentials] = None


def default_state_root(environ: Optional[Mapping[str, str]] = None) -> str:
    environ = os.environ if environ is None else environ
    root = environ.get("TPI_STATE_ROOT")
    if root:
        return root
    base = environ.get("XDG_STATE_HOME") or os.path.join(
        environ.get("HOME") or "/tmp", ".local", "state")
    return os.path.join(base, "tpi")


@record
class Cloud:
    provider: str = PROVIDER_LOCAL
    region: str = "us-west"
    timeouts: Timeouts = field(default_factory=Timeouts)
    credentials: Credentials = field(default_factory=Credentials)
    tags: Dict[str, str] = field(default_factory=dict)

    def state_root(self) -> str:
        if self.credentials.node and self.credentials.node.state_root:
            return self.credentials.node.state_root
        return default_state_root()

    def get_closest_region(self, regions: Mapping[str, str]) -> str:
        """``cloud.go:61-69``: reverse lookup of a native region in an alias map."""
        for key, value in regions.items():
            if value == self.region:
                return key
        raise KeyError("native region not found")


def parse_region_selectors(region: str) -> Dict[str, str]:
    """``k=v,k2=v2`` selector list (``resource_job.go:41-46``); other tokens ignored."""
    selectors: Dict[str, str] = {}
    for item in (region or "").split(","):
        key, sep, value = item.partition("=")
        if sep and value:
            selectors[key.strip()] = value.strip()
    return selectors
