"""Task factory (reference: ``task/task.go:17-45``)."""
from __future__ import annotations

import os
from ..utils.record import replace
from typing import List

from ..models.cloud import (ALL_PROVIDERS, NODE_PROVIDERS, REMOTE_PROVIDERS, Cloud)
from ..models.values import RemoteStorage, Task as TaskSpec
from ..utils.identifier import Identifier
from .base import Resource, Task
from .node import NodeTask, list_tasks as _node_list
from .remote import RemoteProviderUnavailable, RemoteTask, list_tasks as _remote_list
from .ssh import RemoteNodeTask, is_remote, list_tasks as _ssh_list


class UnknownProviderError(ValueError):
    def __init__(self, provider: str):
        super().__init__("unknown provider: %r (expected one of %s)"
                         % (provider, ", ".join(ALL_PROVIDERS)))


def _retarget(cloud: Cloud) -> Cloud:
    """``TPI_REMOTE_AS=mi355x|local`` runs configurations written for a remote cloud on a
    node runtime; with ``TPI_REMOTE_HOST=[user@]node`` on that node over SSH (the cloud's own
    region names no node, so it is replaced by ``host=...``)."""
    target = os.environ.get("TPI_REMOTE_AS")
    if cloud.provider in REMOTE_PROVIDERS and target in NODE_PROVIDERS:
        host = os.environ.get("TPI_REMOTE_HOST")
        if host:
            return replace(cloud, provider=target, region="host=" + host)
        return replace(cloud, provider=target)
    return cloud


# A remote cloud's ``storage.container`` names one of its buckets (``ExistingS3Bucket``,
# ``ExistingBucket``, ``ExistingBlobContainer``: task/{aws,gcp,az}/task.go); run on a node
# runtime, the same bucket is reached over its object-store protocol (storage/objectstore.py).
_BUCKET_SCHEMES = {"aws": "s3", "gcp": "gs", "az": "az"}


def _bucket_container(provider: str, task: TaskSpec) -> TaskSpec:
    rs = task.remote_storage
    scheme = _BUCKET_SCHEMES.get(provider)
    if rs is None or not scheme or not rs.container or "://" in rs.container \
            or rs.container.startswith((":", "/", ".", "~")):
        return task
    return replace(task, remote_storage=RemoteStorage("%s://%s" % (scheme, rs.container),
                                                      rs.path, dict(rs.config)))


def new(cloud: Cloud, identifier: Identifier, task: TaskSpec) -> Task:
    retargeted = _retarget(cloud)
    if retargeted is not cloud:
        task = _bucket_container(cloud.provider, task)
    cloud = retargeted
    if cloud.provider in NODE_PROVIDERS:
        if is_remote(cloud):  # region = "host=...": the node runtime of another host
            return RemoteNodeTask(cloud, identifier, task)
        return NodeTask(cloud, identifier, task)
    if cloud.provider in REMOTE_PROVIDERS:
        return RemoteTask(cloud, identifier, task)
    raise UnknownProviderError(cloud.provider)


def list_tasks(cloud: Cloud) -> List[Identifier]:
    cloud = _retarget(cloud)
    if cloud.provider in NODE_PROVIDERS:
        return _ssh_list(cloud) if is_remote(cloud) else _node_list(cloud)
    if cloud.provider in REMOTE_PROVIDERS:
        return _remote_list(cloud)
    raise UnknownProviderError(cloud.provider)


__all__ = ["new", "list_tasks", "Task", "Resource", "NodeTask", "RemoteTask", "RemoteNodeTask",
           "RemoteProviderUnavailable", "UnknownProviderError"]
