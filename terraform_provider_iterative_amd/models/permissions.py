"""``permission_set`` grammar per cloud (the reference's PermissionSet data sources).

* aws  — IAM instance-profile ARN (``task/aws/resources/data_source_permission_set.go:14-41``)
* az   — comma-separated user-assigned identity ARM ids
         (``task/az/resources/data_source_permission_set.go:16-61``)
* gcp  — ``email,scopes=a,b`` with scope aliases
         (``task/gcp/resources/data_source_permission_set.go:14-96``)
* k8s  — a service account name (``task/k8s/resources/data_source_permission_set.go``)
* local / mi355x — recorded only: ranks run as the invoking user on the node.

Errors carry the reference's messages so configurations fail the same way.
"""
from __future__ import annotations

import json
import re
from typing import Any, Dict, Optional

_AWS_ARN = re.compile(r"arn:aws:iam::[\d]*:instance-profile/[\S]*")
_AZ_ARM_ID = re.compile(r"^/subscriptions/(\w{8}-\w{4}-\w{4}-\w{4}-\w{12})/resourceGroups/(.*)"
                        r"/providers/Microsoft.ManagedIdentity/userAssignedIdentities/(.*)")

GCP_SCOPES = {
    "bigquery": "https://www.googleapis.com/auth/bigquery",
    "cloud-platform": "https://www.googleapis.com/auth/cloud-platform",
    "cloud-source-repos": "https://www.googleapis.com/auth/source.full_control",
    "cloud-source-repos-ro": "https://www.googleapis.com/auth/source.read_only",
    "compute-ro": "https://www.googleapis.com/auth/compute.readonly",
    "compute-rw": "https://www.googleapis.com/auth/compute",
    "datastore": "https://www.googleapis.com/auth/datastore",
    "logging-write": "https://www.googleapis.com/auth/logging.write",
    "monitoring": "https://www.googleapis.com/auth/monitoring",
    "monitoring-read": "https://www.googleapis.com/auth/monitoring.read",
    "monitoring-write": "https://www.googleapis.com/auth/monitoring.write",
    "pubsub": "https://www.googleapis.com/auth/pubsub",
    "service-control": "https://www.googleapis.com/auth/servicecontrol",
    "service-management": "https://www.googleapis.com/auth/service.management.readonly",
    "sql": "https://www.googleapis.com/auth/sqlservice",
    "sql-admin": "https://www.googleapis.com/auth/sqlservice.admin",
    "storage-full": "https://www.googleapis.com/auth/devstorage.full_control",
    "storage-ro": "https://www.googleapis.com/auth/devstorage.read_only",
    "storage-rw": "https://www.googleapis.com/auth/devstorage.read_write",
    "taskqueue": "https://www.googleapis.com/auth/taskqueue",
    "trace": "https://www.googleapis.com/auth/trace.append",
    "useraccounts-ro": "https://www.googleapis.com/auth/cloud.useraccounts.readonly",
    "useraccounts-rw": "https://www.googleapis.com/auth/cloud.useraccounts",
    "userinfo-email": "https://www.googleapis.com/auth/userinfo.email",
}


class PermissionSetError(ValueError):
    pass


def validate_arm_id(identity: str) -> None:
    if not _AZ_ARM_ID.match(identity):
        # Go's %q quoting (json.dumps matches it for printable ASCII)
        raise PermissionSetError("invalid user-assigned identity id: %s" % json.dumps(identity))


def parse_permission_set(provider: str, value: str) -> Optional[Dict[str, Any]]:
    """Normalised permission set (``None`` when empty); raises :class:`PermissionSetError`."""
    if not value:
        return None
    if provider == "aws":
        if not _AWS_ARN.search(value):
            raise PermissionSetError("invalid IAM Instance Profile: %s" % value)
        return {"arn": value}
    if provider == "az":
        identities = []
        for identity in value.split(","):
            identity = identity.strip()
            if not identity:
                continue
            validate_arm_id(identity)
            identities.append(identity)
        return {"user_assigned_identities": identities} if identities else None
    if provider == "gcp":
        parts = value.split(",")
        if len(parts) == 1:
            raise PermissionSetError("at least one scope is required")
        first = parts[1].split("=")
        if len(first) < 2:
            raise PermissionSetError("scopes must be given as scopes=a,b,...")
        scopes = [first[1]] + parts[2:]
        return {"email": parts[0], "scopes": [GCP_SCOPES.get(s, s) for s in scopes]}
    if provider == "k8s":
        return {"service_account": value}
    return {"recorded": value}
