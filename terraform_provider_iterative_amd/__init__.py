"""MI355X-native task orchestrator with the capabilities and user surface of
terraform-provider-iterative (TPI).

Layers (see docs/ARCHITECTURE.md):

* user surfaces  ``cli.leo`` (``bin/leo``), ``cli.tf`` (``bin/tpi``, Terraform-compatible
  engine) and ``provider.server`` (``bin/terraform-provider-iterative``, tfplugin5 plugin)
* resources      ``provider.resources`` (iterative_task / iterative_machine /
  iterative_cml_runner) over ``models`` (values, schemas, machine types)
* backends       ``backends.node`` (cloud = "local" | "mi355x") and ``backends.remote``
* node runtime   ``csrc/supervisor`` (native rank supervisor), ``parallel.placement``
  (reservations of GPUs, cores and memory; the node queue; spot reclaim),
  ``parallel.scheduler`` (queue waiter), ``storage`` (rclone-compatible sync, native walker)
* data plane     ``ops`` + ``checkpoint`` + ``runtime`` (stager, workdir) + ``parallel.comm``:
  hand-written CDNA4 HIP kernels (CRC32C tiles, XXH64 shard hashes, pack/unpack),
  pinned-host checkpoint pipeline, HBM workdir staging, RCCL fan-out over xGMI
"""

from ._version import __version__

__all__ = ["__version__"]
