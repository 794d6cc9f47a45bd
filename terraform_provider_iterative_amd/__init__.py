"""MI355X-native task orchestrator with the capabilities and user surface of
terraform-provider-iterative (TPI).

Layers (see docs/ARCHITECTURE.md):

* user surfaces  ``cli.leo`` (``bin/leo``), ``cli.tf`` (``bin/tpi``, Terraform-compatible
  engine) and ``provider.server`` (``bin/terraform-provider-iterative``, tfplugin5 plugin)
* resources      ``provider.resources`` (iterative_task / iterative_machine /
  iterative_cml_runner) over ``models`` (values, schemas, machine types)
* backends       ``backends.node`` (cloud = "local" | "mi355x") and ``backends.remote``
* node runtime   ``csrc/supervisor`` (native rank supervisor), ``parallel.placement``
  (GPU leases), ``storage`` (rclone-compatible sync, native walker)
* data plane     ``ops`` + ``checkpoint`` + ``runtime.workdir`` + ``parallel.broadcast``:
  hand-written CDNA4 HIP kernels (CRC32C tiles, XXH64 shard hashes, pack/unpack),
  pinned-host checkpoint pipeline, HBM workdir staging, RCCL fan-out over xGMI
"""

from ._version import __version__

__all__ = ["__version__"]
