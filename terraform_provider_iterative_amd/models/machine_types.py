"""Machine types: generic aliases, per-cloud catalogs and the node-local grammar.

Reference catalogs: ``resource_launch_template.go:60-73`` (aws), ``resource_virtual_machine_
scale_set.go:111-123`` (az), ``resource_instance_template.go:72-84`` (gcp),
``resource_job.go:71-126`` (k8s grammar ``cpu-memMB[+acc*n]``); documented in
``docs/guides/generic-machine-types.md``.

On the node-local providers a machine is ``cpus``, ``memory_mb`` and ``gpus`` MI355X GPUs.
Aliases: ``s m l xl`` (CPU only), ``m+mi355x`` (1 GPU), ``l+mi355x`` (4), ``xl+mi355x`` (8);
the reference's GPU aliases map to the same GPU counts (``m+v100`` -> 1, ``l+v100`` -> 4,
``xl+v100`` -> 8, ...), and the explicit form is ``{cpu}-{memMB}+mi355x*{n}``.
"""
from __future__ import annotations

import re
from typing import Dict, Optional

from ..utils.record import record

GENERIC = ("s", "m", "l", "xl", "m+t4", "m+k80", "l+k80", "xl+k80", "m+v100", "l+v100",
           "xl+v100")

CLOUD_CATALOG: Dict[str, Dict[str, str]] = {
    "aws": {"s": "t2.micro", "m": "m5.2xlarge", "l": "m5.8xlarge", "xl": "m5.16xlarge",
            "m+t4": "g4dn.xlarge", "m+k80": "p2.xlarge", "l+k80": "p2.8xlarge",
            "xl+k80": "p2.16xlarge", "m+v100": "p3.xlarge", "l+v100": "p3.8xlarge",
            "xl+v100": "p3.16xlarge"},
    "az": {"s": "Standard_B1s", "m": "Standard_F8s_v2", "l": "Standard_F32s_v2",
           "xl": "Standard_F64s_v2", "m+t4": "Standard_NC4as_T4_v3", "m+k80": "Standard_NC6",
           "l+k80": "Standard_NC12", "xl+k80": "Standard_NC24", "m+v100": "Standard_NC6s_v3",
           "l+v100": "Standard_NC12s_v3", "xl+v100": "Standard_NC24s_v3"},
    "gcp": {"s": "g1-small", "m": "e2-custom-8-32768", "l": "e2-custom-32-131072",
            "xl": "n2-custom-64-262144", "m+t4": "n1-standard-4+nvidia-tesla-t4*1",
            "m+k80": "custom-8-53248+nvidia-tesla-k80*1",
            "l+k80": "custom-32-131072+nvidia-tesla-k80*4",
            "xl+k80": "custom-64-212992-ext+nvidia-tesla-k80*8",
            "m+v100": "custom-8-65536-ext+nvidia-tesla-v100*1",
            "l+v100": "custom-32-262144-ext+nvidia-tesla-v100*4",
            "xl+v100": "custom-64-524288-ext+nvidia-tesla-v100*8"},
    "k8s": {"s": "1-1000", "m": "8-32000", "l": "32-128000", "xl": "64-256000",
            "m+t4": "4-16000+nvidia*1", "m+k80": "4-64000+nvidia*1",
            "l+k80": "32-512000+nvidia*8", "xl+k80": "64-768000+nvidia*16",
            "m+v100": "8-64000+nvidia*1", "l+v100": "32-256000+nvidia*4",
            "xl+v100": "64-512000+nvidia*8"},
}

# Node-local catalog, k8s grammar.
NODE_CATALOG: Dict[str, str] = {
    "s": "1-1000", "m": "8-32000", "l": "32-128000", "xl": "64-256000",
    "m+mi355x": "16-256000+mi355x*1", "l+mi355x": "64-1024000+mi355x*4",
    "xl+mi355x": "128-2048000+mi355x*8",
    # the reference's GPU aliases keep their GPU counts
    "m+t4": "4-16000+mi355x*1", "m+k80": "4-64000+mi355x*1", "l+k80": "32-512000+mi355x*8",
    "m+v100": "8-64000+mi355x*1", "l+v100": "32-256000+mi355x*4",
    "xl+v100": "64-512000+mi355x*8",
}

GPU_ACCELERATORS = ("mi355x", "mi355", "gpu", "amd", "amd.com/gpu", "nvidia", "instinct")
_GRAMMAR = re.compile(r"^(\d+)-(\d+)(?:\+([^*]+)\*([1-9]\d*))?$")
MAX_GPUS_PER_NODE = 8


class MachineTypeError(ValueError):
    pass


@record(frozen=True)
class MachineType:
    name: str
    cpus: int
    memory_mb: int
    gpus: int = 0
    accelerator: str = ""

    def grammar(self) -> str:
        base = "%d-%d" % (self.cpus, self.memory_mb)
        return base + ("+%s*%d" % (self.accelerator or "mi355x", self.gpus) if self.gpus else "")


def parse_node_machine(machine: str, max_gpus: int = MAX_GPUS_PER_NODE) -> MachineType:
    """Resolve a ``machine`` value for the ``local``/``mi355x`` providers."""
    name = (machine or "m").strip()
    spec = NODE_CATALOG.get(name, name)
    match = _GRAMMAR.match(spec)
    if not match:
        raise MachineTypeError(
            "invalid machine type %r: use one of %s or {cpu}-{memMB}[+mi355x*{n}]"
            % (machine, ", ".join(sorted(NODE_CATALOG))))
    cpus, mem = int(match.group(1)), int(match.group(2))
    acc, count = match.group(3) or "", int(match.group(4) or 0)
    if acc and acc.lower() not in GPU_ACCELERATORS:
        raise MachineTypeError("unsupported accelerator %r (this node has MI355X GPUs)" % acc)
    if count > max_gpus:
        raise MachineTypeError("%r asks for %d GPUs; one node has %d" % (machine, count, max_gpus))
    return MachineType(name=name, cpus=cpus, memory_mb=mem, gpus=count,
                       accelerator="mi355x" if count else "")


def cloud_machine(provider: str, machine: str) -> str:
    """Native machine type a remote provider would use for a generic alias."""
    return CLOUD_CATALOG.get(provider, {}).get(machine, machine)


def gpus_for(machine: Optional[str]) -> int:
    return parse_node_machine(machine or "m").gpus
