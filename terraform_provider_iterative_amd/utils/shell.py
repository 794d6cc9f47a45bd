"""Shell quoting with the semantics of ``alessio/shellescape`` used by the reference
(``task/common/machine/script.go``, ``cmd/leo/create/create.go:77-81``)."""
from __future__ import annotations

import re
from typing import Iterable

_SAFE = re.compile(r"^[\w@%+=:,./-]+$", re.ASCII)


def quote(value: str) -> str:
    if value == "":
        return "''"
    if _SAFE.match(value):
        return value
    return "'" + value.replace("'", "'\"'\"'") + "'"


def quote_command(args: Iterable[str]) -> str:
    return " ".join(quote(a) for a in args)
