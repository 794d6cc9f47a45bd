"""Names of object-store containers (``s3://``, ``gs://``, ``az://`` and rclone's
``:backend,opts:bucket/prefix`` forms): parsing and describing them without the HTTP clients.

Split from :mod:`storage.objectstore` so that every ``tpi apply`` -- which asks "is this
container an object store?" -- does not import ``http.client``, ``ssl``, ``xml.etree`` and
``email.utils`` (~28 ms at start-up, the first half of the apply->first-log metric) unless a
task actually names one.  The connection strings follow rclone's
(``task/common/machine/storage.go:236-263``).
"""
from __future__ import annotations

import posixpath
import re
from typing import Dict, Optional

from .transfer import Connection

# rclone backend name -> canonical name; URL scheme -> canonical name
BACKENDS = {"s3": "s3", "googlecloudstorage": "googlecloudstorage", "gcs": "googlecloudstorage",
            "azureblob": "azureblob"}
SCHEMES = {"s3": "s3", "gs": "googlecloudstorage", "az": "azureblob"}


# -- connection strings --------------------------------------------------------------------------

def parse(container: str, path: str = "", opts: Optional[Dict[str, str]] = None
          ) -> Optional[Connection]:
    """The object-store :class:`Connection` named by a ``storage.container`` value (None: not
    an object store).  ``container`` = bucket, ``path`` = key prefix (no leading ``/``)."""
    conn = None
    m = re.match(r"^(s3|gs|az)://([^/]+)(/.*)?$", container or "")
    if m:
        conn = Connection(SCHEMES[m.group(1)], m.group(2), (m.group(3) or "").strip("/"), {})
    elif (container or "").startswith(":"):
        parsed = Connection.parse(container)
        if parsed.backend in BACKENDS:
            bucket, _, prefix = parsed.container.strip("/").partition("/")
            conn = Connection(BACKENDS[parsed.backend], bucket, prefix.strip("/"),
                              dict(parsed.config))
    if conn is None or not conn.container:
        return None
    for key, value in (opts or {}).items():
        if key != "root" and value is not None and str(value) != "":
            conn.config[str(key)] = str(value)
    if path:
        conn.path = posixpath.join(conn.path, path.strip("/")) if conn.path else path.strip("/")
    conn.path = posixpath.normpath(conn.path).lstrip("/") if conn.path else ""
    if conn.path == ".":
        conn.path = ""
    return conn


def is_object_store(value: str) -> bool:
    if not value:
        return False
    if re.match(r"^(s3|gs|az)://[^/]+", value):
        return True
    return value.startswith(tuple(":%s%s" % (b, sep) for b in BACKENDS for sep in (",", ":")))


def describe(conn: Connection) -> str:
    """``backend://bucket/prefix`` -- a connection without its secrets, for logs and events."""
    scheme = {v: k for k, v in SCHEMES.items()}.get(conn.backend, conn.backend)
    return "%s://%s/%s" % (scheme, conn.container, conn.path) if conn.path else \
        "%s://%s" % (scheme, conn.container)
