"""CML runner readiness from logs (reference: ``iterative/utils/runner.go:10-40``)."""
from __future__ import annotations

import json
import re

_JSON = re.compile(r"\{.+\}")


def parse_log_event(text: str) -> dict:
    return json.loads(text)


def has_status(logs: str, status: str) -> bool:
    """True if any log line carries a JSON record whose ``status`` equals ``status``."""
    for line in logs.splitlines():
        match = _JSON.search(line)
        if not match:
            continue
        try:
            event = parse_log_event(match.group(0))
        except ValueError:
            continue
        if isinstance(event, dict) and event.get("status") == status:
            return True
    return False
