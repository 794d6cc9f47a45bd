#!/usr/bin/env python3
"""Per-direction copy phases of a rocprofv3 run (``--memory-copy-trace`` rocpd database).

The chunk copies (>= 16 MiB) of each direction are split into phases at idle gaps longer than
50 ms (bench.py: warmup + timed overlapped steps, then the sequential and codec-free side
measurements).  Per phase: time span, GB moved, GB/s over the span and while busy, idle gaps
between consecutive copies, chunk copy durations, and the rate of the first vs second half
(a restore that trails its save speeds up in the second half, once the save has finished).

    python scripts/exp/copy_timeline.py gpurun_out/prof_x/prof_results.db [...]
"""
from __future__ import annotations

import sqlite3
import sys


def quantile(values, f):
    return values[min(len(values) - 1, int(f * len(values)))] if values else 0


def phases(copies, gap_ns=50e6):
    out, cur = [], [copies[0]]
    for c in copies[1:]:
        if c[0] - cur[-1][1] > gap_ns:
            out.append(cur)
            cur = [c]
        else:
            cur.append(c)
    out.append(cur)
    return out


def rate(part):
    span = (part[-1][1] - part[0][0]) / 1e9
    return sum(z for _, _, z in part) / 1e9 / span if span > 0 else 0.0


def main(path: str) -> None:
    c = sqlite3.connect(path)
    rows = list(c.execute(
        "select src_agent_type, dst_agent_type, start, end, size from memory_copies "
        "where size >= 16777216 order by start"))
    if not rows:
        print("no chunk copies in %s" % path)
        return
    t_origin = rows[0][2]
    print("| direction | phase | t (s) | chunks | GB | GB/s over span | GB/s busy | idle gaps ms "
          "(p50 / p90 us) | chunk ms p10/p50/p90 | GB/s 1st / 2nd half |")
    print("|---|---:|---|---:|---:|---:|---:|---|---|---|")
    for d in ("GPU->CPU", "CPU->GPU"):
        cp = [(s, e, z) for a, b, s, e, z in rows if "%s->%s" % (a, b) == d]
        if not cp:
            continue
        for i, p in enumerate(phases(cp)):
            tot = sum(z for _, _, z in p)
            busy = sum(e - s for s, e, _ in p) / 1e9
            gaps = sorted(p[j + 1][0] - p[j][1] for j in range(len(p) - 1))
            durs = sorted((e - s) / 1e6 for s, e, _ in p)
            half = len(p) // 2
            print("| %s | %d | %.2f-%.2f | %d | %.1f | %.1f | %.1f | %.1f (%.0f / %.0f) | "
                  "%.2f / %.2f / %.2f | %s |" % (
                      d, i, (p[0][0] - t_origin) / 1e9, (p[-1][1] - t_origin) / 1e9, len(p),
                      tot / 1e9, rate(p), tot / 1e9 / busy if busy else 0, sum(gaps) / 1e6,
                      quantile(gaps, .5) / 1e3, quantile(gaps, .9) / 1e3,
                      quantile(durs, .1), quantile(durs, .5), quantile(durs, .9),
                      "%.1f / %.1f" % (rate(p[:half]), rate(p[half:])) if half > 1 else "-"))


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print("\n`%s`\n" % p)
        main(p)
