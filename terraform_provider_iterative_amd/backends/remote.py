"""The reference's remote clouds (``task/{aws,az,gcp,k8s}``) on the node-local runtime.

BASELINE.json collapses the four cloud backends into one on-node runtime, so configurations
naming them still parse (schemas, machine catalogs, region aliases are kept in
``models/``) but every operation fails with a diagnostic that names the replacement, rather
than the reference's generic ``unknown provider`` error (``task/task.go:17-45``).
``TPI_REMOTE_AS=mi355x|local`` re-targets them onto a node provider instead (handy for
running an unchanged ``main.tf`` written for ``cloud = "aws"`` on this node), and
``TPI_REMOTE_HOST=[user@]node`` onto *another* node's runtime over SSH (``backends/ssh.py``):
the reference's remote workflow with an existing MI355X node in place of a provisioned VM.
"""
from __future__ import annotations

from typing import List

from ..models.cloud import Cloud
from ..models.values import Task as TaskSpec
from ..utils.identifier import Identifier
from .base import Task

REGION_ALIASES = {
    "aws": {"us-east": "us-east-1", "us-west": "us-west-1", "eu-north": "eu-north-1",
            "eu-west": "eu-west-1"},
    "az": {"us-east": "eastus", "us-west": "westus2", "eu-north": "northeurope",
           "eu-west": "westeurope"},
    "gcp": {"us-east": "us-east1-c", "us-west": "us-west1-b", "eu-north": "europe-north1-a",
            "eu-west": "europe-west1-d"},
}


class RemoteProviderUnavailable(RuntimeError):
    def __init__(self, provider: str):
        super().__init__(
            "cloud %r is a remote provider; this framework runs tasks on the node it is "
            "installed on: use cloud = \"mi355x\" (GPUs) or cloud = \"local\" (CPU), or set "
            "TPI_REMOTE_AS=mi355x to run %r configurations here (TPI_REMOTE_HOST=node: on "
            "that node over SSH)" % (provider, provider))


class RemoteTask(Task):
    def __init__(self, cloud: Cloud, identifier: Identifier, task: TaskSpec):
        from ..models.permissions import parse_permission_set

        self.cloud = cloud
        self.identifier = identifier
        self.task = task
        # configuration errors first, with the reference's messages
        parse_permission_set(cloud.provider, task.permission_set or "")

    def _fail(self, *_args, **_kwargs):
        raise RemoteProviderUnavailable(self.cloud.provider)

    read = create = delete = start = stop = push = pull = _fail
    status = events = logs = get_addresses = get_key_pair = _fail

    def get_identifier(self) -> Identifier:
        return self.identifier


def native_region(provider: str, region: str) -> str:
    return REGION_ALIASES.get(provider, {}).get(region, region)


def list_tasks(cloud: Cloud) -> List[Identifier]:
    raise RemoteProviderUnavailable(cloud.provider)
