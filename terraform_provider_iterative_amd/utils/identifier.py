"""Task identifiers, bit-compatible with the reference.

Reference: ``task/common/identifier.go:16-115`` (format ``tpi-{name}-{salt8}-{check8}``,
``hash(seed, n)`` = first ``n`` base36 digits of the SHA-256 digest read as a big-endian
integer, name normalised to ``[a-z0-9-]`` and truncated to 28 characters).  The golden
vectors of ``identifier_test.go:41-74`` are pinned in ``tests/test_common.py``.
"""
from __future__ import annotations

import os
import re

try:  # the builtin module: hashlib would load OpenSSL (~4 ms of every CLI start)
    from _sha256 import sha256 as _sha256
except ImportError:  # pragma: no cover
    from hashlib import sha256 as _sha256

from .record import record
from .petname import generate as _petname

DEFAULT_PREFIX = "tpi"
MAXIMUM_LONG_LENGTH = 50
SHORT_LENGTH = 16
NAME_LENGTH = MAXIMUM_LONG_LENGTH - SHORT_LENGTH - len("tpi---")  # 28

_B36 = "0123456789abcdefghijklmnopqrstuvwxyz"
_PARSE_RE = re.compile(
    r"^([a-z0-9]{3})-([a-z0-9]+(?:[a-z0-9-]*[a-z0-9])?)-([a-z0-9]+)-([a-z0-9]+)$", re.S)
_NON_ALNUM = re.compile(r"[^a-z0-9]+")


class WrongIdentifierError(ValueError):
    """Raised when a string is not a valid identifier (``ErrWrongIdentifier``)."""

    def __init__(self, value: str = ""):
        super().__init__(f"wrong identifier: {value!r}")


def _base36(number: int) -> str:
    if number == 0:
        return "0"
    digits = []
    while number:
        number, rem = divmod(number, 36)
        digits.append(_B36[rem])
    return "".join(reversed(digits))


def _hash(seed: str, size: int) -> str:
    """Deterministic base36 digest (``identifier.go:88-101``)."""
    digest = _sha256(seed.encode("utf-8")).digest()
    result = _base36(int.from_bytes(digest, "big"))
    if len(result) < size:  # pragma: no cover - 2**256 has 50 base36 digits
        raise ValueError("not enough bytes to satisfy requested size")
    return result[:size]


def normalize(identifier: str, truncate: int) -> str:
    """RFC1123-like normalisation (``identifier.go:103-115``)."""
    normalized = _NON_ALNUM.sub("-", identifier.lower())
    if len(normalized) > truncate:
        normalized = normalized[:truncate]
    if normalized.startswith("-"):
        normalized = normalized[1:]
    if normalized.endswith("-"):
        normalized = normalized[:-1]
    return normalized


@record(frozen=True)
class Identifier:
    prefix: str
    name: str
    salt: str

    def long(self) -> str:
        name = normalize(self.name, NAME_LENGTH)
        return f"{self.prefix}-{name}-{self.salt}-{_hash(name + self.salt, SHORT_LENGTH // 2)}"

    def short(self) -> str:
        parts = self.long().split("-")
        return parts[-2] + parts[-1]

    def __str__(self) -> str:  # pragma: no cover - convenience
        return self.long()


def parse_identifier(identifier: str) -> Identifier:
    match = _PARSE_RE.match(identifier or "")
    if match and _hash(match.group(2) + match.group(3), SHORT_LENGTH // 2) == match.group(4):
        return Identifier(prefix=match.group(1), name=match.group(2), salt=match.group(3))
    raise WrongIdentifierError(identifier)


def new_deterministic_identifier(name: str, prefix: str = DEFAULT_PREFIX) -> Identifier:
    seed = normalize(name, NAME_LENGTH)
    return Identifier(prefix=prefix[:3], name=name, salt=_hash(seed, SHORT_LENGTH // 2))


def new_random_identifier(name: str = "", prefix: str = DEFAULT_PREFIX) -> Identifier:
    seed = _base36(int.from_bytes(os.urandom(8), "big"))
    if not name:
        name = _petname(3, "-")
    return Identifier(prefix=prefix[:3], name=name, salt=_hash(seed, SHORT_LENGTH // 2))
