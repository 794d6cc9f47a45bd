"""``TPI [LEVEL]`` log formatting (reference: ``iterative/utils/logger.go:25-104``).

The reference pads each line so Terraform's own ``provider.terraform-provider-iterative:``
prefix is overwritten (``\\r`` trick) and renders three special messages from the resource
data: ``instance``, ``status`` and ``logs``.
"""
from __future__ import annotations

import datetime as _dt
import logging
import re
from typing import Any, Dict, List, Mapping, Optional

COLORS = {"DEBUG": 34, "INFO": 36, "WARNING": 33, "ERROR": 31, "FATAL": 31, "SUCCESS": 32,
          "foreground": 35}
_ANSI = re.compile(r"\x1b\[[0-9;]*m")


def strip_ansi(text: str) -> str:
    return _ANSI.sub("", text)


def hide_unwanted_prefix(level: str, new_prefix: str, message: str,
                         now: Optional[_dt.datetime] = None) -> str:
    now = now or _dt.datetime.now().astimezone()
    time_string = now.strftime("%Y-%m-%dT%H:%M:%S.") + "%03d" % (now.microsecond // 1000) + \
        now.strftime("%z")
    unwanted = len("%s [%s] provider.terraform-provider-iterative: [%s]" % (time_string, level,
                                                                          level))
    out = []
    for line in message.split("\n"):
        padding = " " * max(unwanted - len(strip_ansi(line)), 0)
        out.append("[%s]\r%s %s%s\n" % (level, new_prefix, line, padding))
    return "".join(out)


def format_instance(d: Mapping[str, Any]) -> str:
    spot = float(d.get("spot", -1) or 0)
    spot_text = "(Spot %f/h)" % spot if spot > 0 else ""
    return "%s %s%s in %s" % (d.get("cloud", ""), d.get("machine", ""), spot_text, d.get("region", ""))


def reduce_status(status: Mapping[str, int], parallelism: int) -> str:
    """queued -> succeeded -> failed -> running; later rules win (logger.go:76-90,
    cmd/leo/read/read.go:149-178)."""
    result = "queued"
    if (status.get("succeeded") or 0) >= parallelism:
        result = "succeeded"
    if (status.get("failed") or 0) > 0:
        result = "failed"
    if (status.get("running") or 0) >= parallelism:
        result = "running"
    return result


def format_status(d: Mapping[str, Any]) -> str:
    state = reduce_status(d.get("status") or {}, int(d.get("parallelism") or 1))
    text = {"queued": ("DEBUG", "queued"), "succeeded": ("SUCCESS", "completed successfully"),
            "failed": ("ERROR", "completed with errors"), "running": ("WARNING", "running")}[state]
    return "\x1b[%dmStatus: %s \x1b[1m•\x1b[0m" % (COLORS[text[0]], text[1])


def format_logs(d: Mapping[str, Any]) -> str:
    logs: List[str] = list(d.get("logs") or [])
    message = ""
    for index, log in enumerate(logs):
        prefix = "\n\x1b[%dmLOG %d >> " % (COLORS["foreground"], index)
        message += ("\n" + log.strip("\n")).replace("\n", prefix).strip("\n")
        if index + 1 < len(logs):
            message += "\n"
    return message


class TpiFormatter(logging.Formatter):
    """logging.Formatter with the reference's layout; a record with ``extra={"d": data}``
    and message ``instance``/``status``/``logs`` renders that resource view."""

    def format(self, record: logging.LogRecord) -> str:
        level = record.levelname.upper()
        message = record.getMessage()
        data: Optional[Dict[str, Any]] = getattr(record, "d", None)
        if data is not None:
            renderers = {"instance": format_instance, "status": format_status,
                         "logs": format_logs}
            if message not in renderers:
                raise ValueError("wrong schema logging mode")
            message = renderers[message](data)
        prefix = "\x1b[%dmTPI [%s]\x1b[0m" % (COLORS.get(level, 0), level)
        return hide_unwanted_prefix(level, prefix, message).rstrip("\n")


class PlainFormatter(logging.Formatter):
    """leo's logrus TextFormatter look: ``LEVEL message`` without timestamps."""

    def format(self, record: logging.LogRecord) -> str:
        level = record.levelname.upper()[:4]
        return "\x1b[%dm%s\x1b[0m %s" % (COLORS.get(record.levelname.upper(), 0), level,
                                         record.getMessage())


def setup(verbose: bool = False, formatter: Optional[logging.Formatter] = None,
          level: Optional[int] = None) -> logging.Logger:
    logger = logging.getLogger("tpi")
    logger.handlers[:] = []
    handler = logging.StreamHandler()
    handler.setFormatter(formatter or PlainFormatter())
    logger.addHandler(handler)
    logger.setLevel(level if level is not None else (logging.DEBUG if verbose else logging.INFO))
    logger.propagate = False
    return logger
