#!/usr/bin/env python3
"""Per-kernel counter summary of rocprofv3 --pmc databases (rocpd ``run_results.db``):
for each kernel (name prefix) and counter, the mean value per dispatch and, for the HBM
counters (FETCH_SIZE / WRITE_SIZE, KB), the achieved GB/s over the dispatch's duration.

    python scripts/pmc_summary.py DB [DB ...] [--match k_stream_hash]
"""
from __future__ import annotations

import re
import sqlite3
import sys
from collections import defaultdict


def short(name: str) -> str:
    m = re.match(r"(?:void )?([A-Za-z_0-9:]+(?:<[^>]*>)?)", name)
    return m.group(1) if m else name[:60]


def main(argv) -> None:
    match = None
    if "--match" in argv:
        i = argv.index("--match")
        match = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    rows = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [(value, ns)]
    for db in argv:
        c = sqlite3.connect(db)
        for name, counter, value, dur in c.execute(
                "select name, counter_name, counter_value, duration from pmc_events"):
            k = short(name)
            if match and match not in k:
                continue
            rows[k][counter].append((float(value), float(dur)))
    print("| kernel | counter | dispatches | mean per dispatch | mean us | GB/s |")
    print("|---|---|---:|---:|---:|---:|")
    for k in sorted(rows):
        for counter in sorted(rows[k]):
            vals = rows[k][counter]
            n = len(vals)
            mean = sum(v for v, _ in vals) / n
            us = sum(d for _, d in vals) / n / 1e3
            gbps = ""
            if counter in ("FETCH_SIZE", "WRITE_SIZE") and us > 0:
                gbps = "%.0f" % (mean * 1024 / (us * 1e3))  # KB per dispatch / s -> GB/s
            print("| `%s` | %s | %d | %.4g | %.1f | %s |" % (k, counter, n, mean, us, gbps))


if __name__ == "__main__":
    main(sys.argv[1:])
