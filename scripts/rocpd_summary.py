#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (``run_results.db``) into markdown.

    python scripts/rocpd_summary.py gpurun_out/prof_bench/run_results.db > profiles/x.md
"""
from __future__ import annotations

import re
import sqlite3
import sys


def short(name: str, width: int = 70) -> str:
    name = re.sub(r"\(.*", "", name) if name.startswith("void at::") else name
    return name if len(name) <= width else name[:width - 3] + "..."


def main(path: str) -> None:
    c = sqlite3.connect(path)
    print("## Kernels (%s)\n" % path)
    print("| kernel | calls | total ms | avg us | grid | wg | VGPR | LDS B |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|")
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), max(grid_x), max(workgroup_x), "
        "max(vgpr_count), max(lds_size) from kernels group by name order by sum(duration) desc")
    for name, n, tot, avg, grid, wg, vgpr, lds in rows:
        print("| `%s` | %d | %.3f | %.1f | %d | %d | %d | %d |" % (
            short(name), n, tot / 1e6, avg / 1e3, grid, wg, vgpr or 0, lds or 0))
    copies = list(c.execute(
        "select src_agent_type, dst_agent_type, count(*), sum(size), sum(duration), "
        "avg(size) from memory_copies group by src_agent_type, dst_agent_type"))
    if copies:
        print("\n## Memory copies\n")
        print("| direction | count | total GB | busy s | GB/s while busy | avg MiB |")
        print("|---|---:|---:|---:|---:|---:|")
        for src, dst, n, size, dur, avg in copies:
            print("| %s->%s | %d | %.2f | %.3f | %.1f | %.1f |" % (
                src, dst, n, size / 1e9, dur / 1e9, size / dur if dur else 0, avg / 2**20))


if __name__ == "__main__":
    main(sys.argv[1])
