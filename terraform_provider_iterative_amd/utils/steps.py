"""Ordered resource steps (reference: ``task/common/steps.go:10-26``)."""
from __future__ import annotations

import logging
import time
from typing import Callable, Iterable, List, Optional

from .record import record

log = logging.getLogger("tpi")


@record
class Step:
    description: str
    action: Callable[[], None]


@record
class StepTiming:
    description: str
    seconds: float


def run_steps(steps: Iterable[Step], timings: Optional[List[StepTiming]] = None) -> None:
    """Run ``steps`` in order, logging ``[i/N] description``; stop at the first error.

    When ``timings`` is given, each completed step appends its wall time to it (the
    per-phase journal used by the latency benchmark).
    """
    steps = list(steps)
    total = len(steps)
    for index, step in enumerate(steps, 1):
        log.info("[%d/%d] %s", index, total, step.description)
        start = time.perf_counter()
        try:
            step.action()
        except Exception as error:
            log.debug("step: %s error: %s", step.description, error)
            raise
        if timings is not None:
            timings.append(StepTiming(step.description, time.perf_counter() - start))
