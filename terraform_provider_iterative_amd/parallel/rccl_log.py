"""What RCCL itself says about a communicator: rank count and the transport of every peer link.

The reference has no collective layer; this module exists so that a multi-GPU
run of this repo's fan-out and benchmark can answer "did RCCL see N ranks, and did it connect
them over xGMI (P2P/IPC) rather than through host shared memory (SHM) or the network?" from
its own record.  RCCL prints that at ``NCCL_DEBUG=INFO`` while it builds its rings and trees:

    host:1234:1250 [0] NCCL INFO comm 0x55d5 rank 0 nRanks 8 nNodes 1 localRanks 8 localRank 0
    host:1234:1250 [0] NCCL INFO Channel 00/0 : 0[2a000] -> 1[3a000] via P2P/IPC comm 0x55d5 nRanks 08
    host:1234:1250 [0] NCCL INFO Channel 01/0 : 0[2a000] -> 7[da000] via SHM/direct/direct

:func:`debug_env` points ``NCCL_DEBUG_FILE`` at one file per process (``%p``) and
:func:`parse` reduces such lines to ``{"nranks", "links": {"0->1": "P2P/IPC", ...},
"transports": {"P2P/IPC": k, ...}, "xgmi_only"}``.
"""
from __future__ import annotations

import glob
import os
import re
from typing import Dict, Iterable, List, Optional

_LINK = re.compile(r"(\d+)\[[0-9a-fA-Fx]*\]\s*->\s*(\d+)\[[0-9a-fA-Fx]*\]\s+via\s+(\S+)")
_NRANKS = re.compile(r"\bn[Rr]anks\s+0*(\d+)")
_RANK = re.compile(r"\bcomm\s+0x[0-9a-fA-F]+\s+rank\s+(\d+)\b")
# transports that ride the GPUs' own links (xGMI on MI355X): P2P in any flavour
_XGMI = ("P2P",)


def debug_env(directory: str, env: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    """Environment that makes RCCL log its topology choices to ``directory/rccl-<pid>.log``
    (INFO level, INIT subsystem only: a few hundred lines per communicator).  Variables the
    caller already set win."""
    env = dict(os.environ if env is None else env)
    os.makedirs(directory, exist_ok=True)
    env.setdefault("NCCL_DEBUG", "INFO")
    env.setdefault("NCCL_DEBUG_SUBSYS", "INIT")
    env.setdefault("NCCL_DEBUG_FILE", os.path.join(directory, "rccl-%p.log"))
    return env


def parse(lines: Iterable[str]) -> Dict:
    """Reduce RCCL INFO lines to rank count and per-link transports (see module doc)."""
    links: Dict[str, str] = {}
    nranks: List[int] = []
    ranks = set()
    for line in lines:
        if "NCCL" not in line and "RCCL" not in line:
            continue
        m = _NRANKS.search(line)
        if m:
            nranks.append(int(m.group(1)))
        m = _RANK.search(line)
        if m:
            ranks.add(int(m.group(1)))
        m = _LINK.search(line)
        if m:
            src, dst, via = int(m.group(1)), int(m.group(2)), m.group(3)
            key = "%d->%d" % (src, dst)
            # a pair can appear once per channel; keep every distinct transport it used
            prev = links.get(key)
            if prev is None:
                links[key] = via
            elif via not in prev.split("+"):
                links[key] = prev + "+" + via
    transports: Dict[str, int] = {}
    for via in links.values():
        for v in via.split("+"):
            transports[v] = transports.get(v, 0) + 1
    return {"nranks": max(nranks) if nranks else None,
            "ranks_seen": sorted(ranks),
            "links": dict(sorted(links.items())),
            "transports": transports,
            "xgmi_only": (all(v.startswith(_XGMI) for v in transports) if transports
                          else None)}


def parse_files(pattern: str) -> Dict:
    """:func:`parse` over every file matching ``pattern`` (e.g. ``<dir>/rccl-*.log``)."""
    lines: List[str] = []
    for path in sorted(glob.glob(pattern)):
        try:
            with open(path, errors="replace") as f:
                lines.extend(f)
        except OSError:
            continue
    out = parse(lines)
    out["files"] = len(glob.glob(pattern))
    return out
