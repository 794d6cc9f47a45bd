"""Node queue waiter: the process that holds a queued task's place until its machine fits.

The reference's scaling group is created with ``desired = parallelism`` even when the cloud
has no capacity; the instances appear when it does (``resource_auto_scaling_group.go:51-106,
188-199``), and ``leo read`` shows ``queued`` meanwhile (``cmd/leo/read/read.go:164-176``).  On
one node, :meth:`..backends.node.NodeTask.create` starts this waiter instead of a supervisor
when :meth:`.placement.Placement.reserve` finds the node busy, and a spot task's supervisor
starts it again after the task was reclaimed by an on-demand one.  It polls the placement
(lease files under one ``flock``), reclaims spot capacity while it is the on-demand head of
the queue, and starts the supervisor once the reservation succeeds.
"""
from __future__ import annotations

import sys
from typing import List, Optional


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) != 1:
        print("usage: scheduler <task root>", file=sys.stderr)
        return 2
    from ..backends.node import NodeTask

    return NodeTask.from_root(argv[0]).run_queued()


if __name__ == "__main__":
    sys.exit(main())
