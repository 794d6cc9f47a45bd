"""Object-store ``storage.container``: Amazon S3 (and S3-compatible stores), Azure Blob Storage
and Google Cloud Storage, spoken directly over HTTP(S).

The reference hands these to rclone's ``s3``, ``azureblob`` and ``googlecloudstorage``
backends (``task/common/machine/storage.go:18-21``; the connection strings of ``:236-263``,
built by ``task/aws/resources/data_source_bucket.go:39-50``,
``task/gcp/resources/data_source_bucket.go:40-41`` and
``task/az/resources/data_source_existing_blob_container.go:32-39`` /
``resource_blob_container.go:81-92``).  A node runtime has no rclone; this module implements
the three wire protocols with the standard library (request signing: AWS Signature V4,
Azure Shared Key, Google service-account JWT with RS256) and offers the same file operations
as the SSH container (:class:`storage.remote.SSHRemote`), so the node backend, the task's
data mirror and ``Checkpointer.persist``/``load`` use any of them unchanged.

Forms of ``storage.container`` (``container_opts`` adds or overrides connection options)::

    s3://bucket/prefix           :s3,region='eu-west-1',endpoint='http://minio:9000':bucket/prefix
    gs://bucket/prefix           :googlecloudstorage,service_account_credentials='{...}':bucket/prefix
    az://container/prefix        :azureblob,account='acct',key='base64':container/prefix

Options (rclone's names): S3 ``access_key_id``, ``secret_access_key``, ``session_token``,
``region``, ``endpoint`` (path-style addressing; else virtual-hosted AWS); Azure ``account``,
``key``, ``sas_url``, ``endpoint``; GCS ``service_account_credentials`` (the JSON),
``service_account_file``, ``token`` (a bearer token), ``endpoint``.  Missing credentials come
from the usual environment (``AWS_*``, ``AZURE_STORAGE_ACCOUNT``/``AZURE_STORAGE_KEY``,
``GOOGLE_APPLICATION_CREDENTIALS``), as rclone's ``env_auth``.

Large files move in parallel parts (S3 multipart upload, Azure Put Block / Put Block List,
ranged GETs everywhere; GCS uploads through one resumable session).  ``TPI_OBJECT_THREADS``
(default 8) requests run at once per transfer, ``TPI_OBJECT_PART_MB`` (default 64) per part.

Neither the build container nor the GPU box reaches a cloud: the protocols are tested against
in-process fakes (``tests/objectstore_fakes.py``) and the AWS Signature V4 examples of the S3
documentation; parity against the live services is unpinned.
"""
from __future__ import annotations

import base64
import datetime
import email.utils
import hashlib
import hmac
import http.client
import json
import logging
import os
import posixpath
import re
import ssl
import threading
import time
import urllib.parse
import xml.etree.ElementTree as ET
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, Dict, Iterable, Iterator, List, Optional, Tuple

from .transfer import Connection, make_filter, transfer_rules
from ..ops import native

log = logging.getLogger("tpi")

from .objectnames import BACKENDS, SCHEMES, describe, is_object_store, parse  # noqa: F401


class ObjectStoreError(OSError):
    pass


def _threads() -> int:
    return max(1, int(os.environ.get("TPI_OBJECT_THREADS", "8")))


def _part_bytes() -> int:
    return max(1, int(os.environ.get("TPI_OBJECT_PART_MB", "64"))) << 20


def open_remote(conn: Connection) -> "ObjectRemote":
    cls = {"s3": S3Remote, "azureblob": AzureRemote,
           "googlecloudstorage": GCSRemote}.get(conn.backend)
    if cls is None:
        raise ValueError("not an object-store connection: %s" % describe(conn))
    return cls(conn)


# -- HTTP ----------------------------------------------------------------------------------------

class _Http:
    """Keep-alive connections (one per thread) to one origin; transient failures (connection
    errors, 5xx, 429) are retried with backoff, each attempt signed anew."""

    RETRIES = 4

    def __init__(self, base_url: str, timeout: float = 600.0):
        u = urllib.parse.urlsplit(base_url)
        if u.scheme not in ("http", "https") or not u.hostname:
            raise ValueError("bad endpoint %r" % base_url)
        self.https = u.scheme == "https"
        self.host, self.port = u.hostname, u.port
        self.netloc = u.netloc
        self.base_path = u.path.rstrip("/")
        self.timeout = timeout
        self.local = threading.local()

    def _conn(self) -> http.client.HTTPConnection:
        c = getattr(self.local, "conn", None)
        if c is None:
            if self.https:
                c = http.client.HTTPSConnection(self.host, self.port, timeout=self.timeout,
                                                context=ssl.create_default_context())
            else:
                c = http.client.HTTPConnection(self.host, self.port, timeout=self.timeout)
            self.local.conn = c
        return c

    def _drop(self) -> None:
        c = getattr(self.local, "conn", None)
        if c is not None:
            c.close()
        self.local.conn = None

    def request(self, method: str, path: str, query: str,
                sign: Callable[[], Dict[str, str]], body: bytes = b"",
                ok: Tuple[int, ...] = (200, 201, 204, 206)) -> Tuple[int, Dict[str, str], bytes]:
        """One request; returns (status, lowercase headers, body).  Statuses outside ``ok``
        (after retries) raise :class:`ObjectStoreError`, except a 404 of a read or a delete
        (returned: callers decide whether a missing object is an error)."""
        url = path + ("?" + query if query else "")
        delay = 0.2
        for attempt in range(self.RETRIES):
            try:
                headers = sign()
                c = self._conn()
                c.request(method, url, body=body if body else None, headers=headers)
                r = c.getresponse()
                data = r.read()
                hdrs = {k.lower(): v for k, v in r.getheaders()}
                if r.will_close:
                    self._drop()
            except (OSError, http.client.HTTPException) as error:
                self._drop()
                if attempt == self.RETRIES - 1:
                    raise ObjectStoreError("%s %s: %s" % (method, path, error))
                time.sleep(delay)
                delay *= 2
                continue
            # a missing object is the caller's call on reads and deletes; a write that finds no
            # bucket / container / upload session has failed
            if r.status in ok or r.status == 308 or (
                    r.status == 404 and method in ("GET", "HEAD", "DELETE")):
                return r.status, hdrs, data
            if (r.status >= 500 or r.status == 429) and attempt < self.RETRIES - 1:
                time.sleep(delay)
                delay *= 2
                continue
            raise ObjectStoreError("%s %s: HTTP %d: %s" % (
                method, path, r.status, data[:500].decode(errors="replace")))
        raise ObjectStoreError("%s %s: out of retries" % (method, path))


def _quote(s: str, safe: str = "/-_.~") -> str:
    return urllib.parse.quote(s, safe=safe)


def _query(params: Dict[str, str]) -> str:
    """Sorted, RFC 3986-encoded query string (the form Signature V4 signs, sent as is)."""
    return "&".join("%s=%s" % (_quote(k, "-_.~"), _quote(str(v), "-_.~"))
                    for k, v in sorted(params.items()))


def _xml_strip(root: ET.Element) -> ET.Element:
    for el in root.iter():
        if isinstance(el.tag, str) and el.tag.startswith("{"):
            el.tag = el.tag.split("}", 1)[1]
    return root


# -- the file operations, on top of a few object primitives ---------------------------------------

class ObjectRemote:
    """File operations on a bucket prefix: the interface of :class:`storage.remote.SSHRemote`
    (``exists``, ``put_tree``, ``get_tree``, ``remove``, ``put_file``, ``get_file``)."""

    def __init__(self, conn: Connection):
        self.conn = conn
        self.bucket = conn.container
        self.root = (conn.path or "").strip("/")
        self.part = _part_bytes()
        self.threads = _threads()
        # part buffers in flight over all the files of one transfer
        self._slots = threading.BoundedSemaphore(2 * self.threads)

    def __str__(self) -> str:
        return describe(self.conn)

    def path(self, *parts: str) -> str:
        """The object key of a path relative to the container's prefix."""
        joined = posixpath.normpath(posixpath.join("/", self.root, *[p.lstrip("/") for p in parts]))
        return joined.lstrip("/")

    # primitives (per protocol) ------------------------------------------------------------------
    def _head(self, key: str) -> Optional[int]:
        raise NotImplementedError

    def _list(self, prefix: str) -> Iterator[Tuple[str, int]]:
        raise NotImplementedError

    def _put(self, key: str, data: bytes, meta: Dict[str, str]) -> None:
        raise NotImplementedError

    def _get(self, key: str, start: int, end: int) -> bytes:
        """Bytes ``[start, end]`` (inclusive) of an object."""
        raise NotImplementedError

    def _delete(self, keys: List[str]) -> None:
        raise NotImplementedError

    def _upload_large(self, key: str, local: str, size: int, meta: Dict[str, str],
                      pool: ThreadPoolExecutor) -> None:
        raise NotImplementedError

    # helpers -------------------------------------------------------------------------------------
    def _read(self, local, offset: int, length: int):
        """``length`` bytes at ``offset`` of a file (path) or of a buffer (memoryview: a
        slice, no copy)."""
        if isinstance(local, memoryview):
            return local[offset:offset + length]
        with open(local, "rb") as f:
            f.seek(offset)
            data = f.read(length)
        if len(data) != length:
            raise ObjectStoreError("%s changed size while it was uploaded" % local)
        return data

    def _upload(self, key: str, local, pool: ThreadPoolExecutor) -> int:
        if isinstance(local, memoryview):
            size, meta = local.nbytes, {"mtime": "%.9f" % time.time()}
        else:
            st = os.stat(local)
            size, meta = st.st_size, {"mtime": "%.9f" % st.st_mtime}
        if size <= self.part:
            with self._slots:
                self._put(key, self._read(local, 0, size), meta)
        else:
            self._upload_large(key, local, size, meta, pool)
        return size

    def _download(self, key: str, size: int, local: str, pool: ThreadPoolExecutor) -> int:
        os.makedirs(os.path.dirname(os.path.abspath(local)), exist_ok=True)
        tmp = local + ".tpi-partial"
        fd = os.open(tmp, os.O_CREAT | os.O_TRUNC | os.O_WRONLY, 0o644)
        try:
            os.ftruncate(fd, size)

            def piece(start: int) -> None:
                end = min(size, start + self.part) - 1
                with self._slots:
                    data = self._get(key, start, end)
                    if len(data) != end - start + 1:
                        raise ObjectStoreError("%s: short read at %d" % (key, start))
                    os.pwrite(fd, data, start)

            starts = list(range(0, size, self.part))
            if len(starts) <= 1:
                for s in starts:
                    piece(s)
            else:
                for fut in [pool.submit(piece, s) for s in starts]:
                    fut.result()
        except BaseException:
            os.close(fd)
            os.remove(tmp)
            raise
        os.close(fd)
        os.replace(tmp, local)
        return size

    def _run(self, jobs: List[Callable[[ThreadPoolExecutor], int]]) -> int:
        """Run file jobs ``threads`` at a time; their part requests use a second pool (no job
        waits on a pool it occupies)."""
        total = 0
        with ThreadPoolExecutor(self.threads, thread_name_prefix="tpi-obj-part") as parts, \
                ThreadPoolExecutor(self.threads, thread_name_prefix="tpi-obj-file") as files:
            for fut in [files.submit(job, parts) for job in jobs]:
                total += fut.result()
        return total

    # the SSHRemote interface ---------------------------------------------------------------------
    def exists(self, rel: str = "") -> bool:
        key = self.path(rel)
        if key and self._head(key) is not None:
            return True
        for _ in self._list(key + "/" if key else ""):
            return True
        return False

    def put_file(self, local: str, rel: str) -> int:
        return self._run([lambda pool: self._upload(self.path(rel), local, pool)])

    def put_bytes(self, data: memoryview, rel: str) -> int:
        """Upload a buffer as one object (a checkpoint slot straight from its host region:
        no temporary file)."""
        return self._run([lambda pool: self._upload(self.path(rel), memoryview(data).cast("B"),
                                                     pool)])

    def get_file(self, rel: str, local: str) -> int:
        key = self.path(rel)
        size = self._head(key)
        if size is None:
            raise FileNotFoundError("%s: no object %s" % (self, key))
        return self._run([lambda pool: self._download(key, size, local, pool)])

    def size(self, rel: str) -> Optional[int]:
        """Bytes of the object at ``rel`` (None: no such object)."""
        return self._head(self.path(rel))

    def read(self, rel: str, offset: int, n: int) -> bytes:
        """``n`` bytes at ``offset`` of an object (one ranged request)."""
        if n <= 0:
            return b""
        with self._slots:
            data = self._get(self.path(rel), offset, offset + n - 1)
        if len(data) != n:
            raise ObjectStoreError("%s: short read of %s at %d" % (self, rel, offset))
        return data

    def read_into(self, rel: str, addr: int, offset: int, n: int,
                  progress: Optional[Callable[[int], None]] = None) -> int:
        """Bytes ``[offset, offset + n)`` of an object into memory at ``addr`` (ranged GETs,
        ``threads`` at once); ``progress(b)`` is called, in order, each time the prefix
        ``[0, b)`` is complete -- a streamed restore runs behind it (Checkpointer.load)."""
        import ctypes

        key = self.path(rel)
        starts = list(range(0, n, self.part))
        done = set()
        lock = threading.Lock()
        state = {"prefix": 0}

        def piece(i: int) -> None:
            a = starts[i]
            b = min(n, a + self.part)
            with self._slots:
                data = self._get(key, offset + a, offset + b - 1)
                if len(data) != b - a:
                    raise ObjectStoreError("%s: short read of %s at %d" % (self, key, offset + a))
                ctypes.memmove(addr + a, data, b - a)
            with lock:
                done.add(i)
                advanced = False
                while state["prefix"] < len(starts) and state["prefix"] in done:
                    state["prefix"] += 1
                    advanced = True
                if advanced and progress is not None:
                    progress(min(n, starts[state["prefix"] - 1] + self.part))

        with ThreadPoolExecutor(self.threads, thread_name_prefix="tpi-obj-read") as pool:
            for fut in [pool.submit(piece, i) for i in range(len(starts))]:
                fut.result()
        return n

    def put_tree(self, local_dir: str, rel: str, rules: Optional[List[str]] = None,
                 only: Optional[Iterable[str]] = None) -> Dict[str, int]:
        """Upload ``local_dir`` (filter ``rules``; ``only``: just these relative paths) under
        ``<prefix>/<rel>`` -- rclone copy semantics: nothing there is deleted."""
        flt = make_filter(transfer_rules([]) if rules is None else rules)
        entries = [e for e in native().walk(local_dir, flt) if not e[4]]
        if only is not None:
            wanted = set(only)
            entries = [e for e in entries if e[0] in wanted]
        jobs = [(lambda pool, r=relpath: self._upload(self.path(rel, r),
                                                      os.path.join(local_dir, r), pool))
                for relpath, _size, _mtime, _mode, _ in entries]
        nbytes = self._run(jobs)
        return {"files": len(entries), "bytes": nbytes}

    def get_tree(self, rel: str, local_dir: str, rules: Optional[List[str]] = None
                 ) -> Dict[str, int]:
        """Download ``<prefix>/<rel>/**`` into ``local_dir`` through filter ``rules`` (nothing
        there: nothing copied)."""
        base = self.path(rel)
        prefix = base + "/" if base else ""
        flt = make_filter(transfer_rules([]) if rules is None else rules)
        wanted = []
        for key, size in self._list(prefix):
            name = posixpath.normpath(key[len(prefix):])
            if key.endswith("/") or name in (".", "") or name.startswith("../") \
                    or name.startswith("/") or not flt.include_file(name):
                continue
            wanted.append((key, size, os.path.join(local_dir, name)))
        os.makedirs(local_dir, exist_ok=True)
        jobs = [(lambda pool, k=k, s=s, t=t: self._download(k, s, t, pool))
                for k, s, t in wanted]
        nbytes = self._run(jobs)
        return {"files": len(wanted), "bytes": nbytes}

    def remove(self, rels: Iterable[str]) -> None:
        keys = [self.path(r) for r in rels]
        if keys:
            self._delete(keys)


# -- Amazon S3 and S3-compatible stores ------------------------------------------------------------

def sigv4_authorization(method: str, canonical_uri: str, canonical_query: str,
                        headers: Dict[str, str], payload_hash: str, region: str, service: str,
                        access_key: str, secret_key: str, amz_date: str) -> str:
    """The ``Authorization`` header of AWS Signature Version 4 over exactly ``headers`` (all of
    them are signed)."""
    canon = {k.lower(): " ".join(str(v).strip().split()) for k, v in headers.items()}
    names = sorted(canon)
    canonical_request = "\n".join([
        method, canonical_uri, canonical_query,
        "".join("%s:%s\n" % (n, canon[n]) for n in names), ";".join(names), payload_hash])
    scope = "%s/%s/%s/aws4_request" % (amz_date[:8], region, service)
    string_to_sign = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope,
                                hashlib.sha256(canonical_request.encode()).hexdigest()])
    key = ("AWS4" + secret_key).encode()
    for part in (amz_date[:8], region, service, "aws4_request"):
        key = hmac.new(key, part.encode(), hashlib.sha256).digest()
    signature = hmac.new(key, string_to_sign.encode(), hashlib.sha256).hexdigest()
    return "AWS4-HMAC-SHA256 Credential=%s/%s,SignedHeaders=%s,Signature=%s" % (
        access_key, scope, ";".join(names), signature)


EMPTY_SHA256 = hashlib.sha256(b"").hexdigest()


class S3Remote(ObjectRemote):
    """S3 REST API with Signature V4 (anonymous when no keys are known).  ``endpoint`` given:
    path-style requests to it (MinIO, Ceph RGW, ...); else virtual-hosted AWS."""

    def __init__(self, conn: Connection):
        super().__init__(conn)
        cfg = conn.config
        env = os.environ
        self.region = cfg.get("region") or env.get("AWS_REGION") or \
            env.get("AWS_DEFAULT_REGION") or "us-east-1"
        self.access = cfg.get("access_key_id") or env.get("AWS_ACCESS_KEY_ID", "")
        self.secret = cfg.get("secret_access_key") or env.get("AWS_SECRET_ACCESS_KEY", "")
        self.token = cfg.get("session_token") or (
            env.get("AWS_SESSION_TOKEN", "") if not cfg.get("access_key_id") else "")
        endpoint = cfg.get("endpoint") or env.get("TPI_S3_ENDPOINT", "")
        if endpoint:
            if "://" not in endpoint:
                endpoint = "https://" + endpoint
            self.http = _Http(endpoint)
            self.prefix_path = self.http.base_path + "/" + _quote(self.bucket, "-_.~")
        elif "." in self.bucket:  # dotted names break the wildcard certificate
            self.http = _Http("https://s3.%s.amazonaws.com" % self.region)
            self.prefix_path = "/" + _quote(self.bucket, "-_.~")
        else:
            self.http = _Http("https://%s.s3.%s.amazonaws.com" % (self.bucket, self.region))
            self.prefix_path = ""

    def _request(self, method: str, key: Optional[str], params: Optional[Dict[str, str]] = None,
                 headers: Optional[Dict[str, str]] = None, body: bytes = b"",
                 ok: Tuple[int, ...] = (200, 201, 204, 206)):
        path = self.prefix_path + "/" + (_quote(key) if key else "")
        query = _query(params or {})
        payload = hashlib.sha256(body).hexdigest() if body else EMPTY_SHA256

        def sign() -> Dict[str, str]:
            h = dict(headers or {})
            if not self.access:
                return h
            amz_date = datetime.datetime.now(datetime.timezone.utc).strftime("%Y%m%dT%H%M%SZ")
            h.update({"host": self.http.netloc, "x-amz-date": amz_date,
                      "x-amz-content-sha256": payload})
            if self.token:
                h["x-amz-security-token"] = self.token
            h["Authorization"] = sigv4_authorization(method, path, query, h, payload,
                                                     self.region, "s3", self.access,
                                                     self.secret, amz_date)
            return h

        return self.http.request(method, path, query, sign, body, ok)

    @staticmethod
    def _check_xml_error(data: bytes, what: str) -> ET.Element:
        root = _xml_strip(ET.fromstring(data))
        if root.tag == "Error":  # S3 may report a failed completion with HTTP 200
            raise ObjectStoreError("%s: %s: %s" % (what, root.findtext("Code"),
                                                   root.findtext("Message")))
        return root

    def _head(self, key: str) -> Optional[int]:
        status, hdrs, _ = self._request("HEAD", key)
        return None if status == 404 else int(hdrs.get("content-length", "0"))

    def _list(self, prefix: str) -> Iterator[Tuple[str, int]]:
        token = None
        while True:
            params = {"list-type": "2", "prefix": prefix}
            if token:
                params["continuation-token"] = token
            status, _, data = self._request("GET", None, params)
            if status == 404:
                raise ObjectStoreError("%s: no bucket %s" % (self, self.bucket))
            root = self._check_xml_error(data, "list")
            for item in root.findall("Contents"):
                yield item.findtext("Key"), int(item.findtext("Size") or 0)
            if root.findtext("IsTruncated") != "true":
                return
            token = root.findtext("NextContinuationToken")

    def _put(self, key: str, data: bytes, meta: Dict[str, str]) -> None:
        headers = {"Content-Type": "application/octet-stream",
                   "Content-MD5": base64.b64encode(hashlib.md5(data).digest()).decode()}
        headers.update({"x-amz-meta-" + k: v for k, v in meta.items()})
        self._request("PUT", key, headers=headers, body=data)

    def _get(self, key: str, start: int, end: int) -> bytes:
        status, _, data = self._request("GET", key, headers={"Range": "bytes=%d-%d" % (start, end)})
        if status == 404:
            raise FileNotFoundError("%s: no object %s" % (self, key))
        return data

    def _upload_large(self, key, local, size, meta, pool) -> None:
        part = max(self.part, -(-size // 10000))  # S3 allows 10000 parts
        headers = {"Content-Type": "application/octet-stream"}
        headers.update({"x-amz-meta-" + k: v for k, v in meta.items()})
        _, _, data = self._request("POST", key, {"uploads": ""}, headers)
        upload_id = self._check_xml_error(data, "multipart upload").findtext("UploadId")
        try:
            def send(index: int) -> str:
                offset = index * part
                with self._slots:
                    body = self._read(local, offset, min(part, size - offset))
                    _, hdrs, _ = self._request(
                        "PUT", key, {"partNumber": str(index + 1), "uploadId": upload_id},
                        {"Content-MD5": base64.b64encode(hashlib.md5(body).digest()).decode()},
                        body)
                return hdrs.get("etag", "")

            etags = [f.result() for f in [pool.submit(send, i)
                                          for i in range(-(-size // part))]]
            body = "<CompleteMultipartUpload>%s</CompleteMultipartUpload>" % "".join(
                "<Part><PartNumber>%d</PartNumber><ETag>%s</ETag></Part>" % (i + 1, e)
                for i, e in enumerate(etags))
            try:
                _, _, data = self._request("POST", key, {"uploadId": upload_id},
                                           body=body.encode())
                self._check_xml_error(data, "complete multipart upload")
            except ObjectStoreError:
                # a completion retried after a lost reply finds its upload gone (NoSuchUpload):
                # the object is there if the first attempt went through
                if self._head(key) != size:
                    raise
        except BaseException:
            try:
                self._request("DELETE", key, {"uploadId": upload_id})
            except ObjectStoreError:
                pass
            raise

    def _delete(self, keys: List[str]) -> None:
        for i in range(0, len(keys), 1000):
            body = ("<Delete><Quiet>true</Quiet>%s</Delete>" % "".join(
                "<Object><Key>%s</Key></Object>" % _xml_escape(k)
                for k in keys[i:i + 1000])).encode()
            _, _, data = self._request(
                "POST", None, {"delete": ""},
                {"Content-MD5": base64.b64encode(hashlib.md5(body).digest()).decode(),
                 "Content-Type": "application/xml"}, body)
            root = self._check_xml_error(data, "delete")
            errors = root.findall("Error")
            if errors:
                raise ObjectStoreError("delete: %s: %s" % (errors[0].findtext("Key"),
                                                           errors[0].findtext("Code")))


def _xml_escape(s: str) -> str:
    return (s.replace("&", "&amp;").replace("<", "&lt;").replace(">", "&gt;")
            .replace('"', "&quot;").replace("'", "&apos;"))


# -- Azure Blob Storage -----------------------------------------------------------------------------

AZURE_VERSION = "2021-08-06"


def azure_shared_key(account: str, key_b64: str, method: str, path: str,
                     params: Dict[str, str], headers: Dict[str, str]) -> str:
    """The ``Authorization`` header of Azure Storage Shared Key authorization (blob service,
    version 2015-02-21 and later: an empty Content-Length when it is 0)."""
    h = {k.lower(): str(v) for k, v in headers.items()}
    length = h.get("content-length", "")
    fields = [method, h.get("content-encoding", ""), h.get("content-language", ""),
              "" if length == "0" else length, h.get("content-md5", ""),
              h.get("content-type", ""), h.get("date", ""), h.get("if-modified-since", ""),
              h.get("if-match", ""), h.get("if-none-match", ""),
              h.get("if-unmodified-since", ""), h.get("range", "")]
    canon_headers = "".join("%s:%s\n" % (k, " ".join(h[k].strip().split()))
                            for k in sorted(h) if k.startswith("x-ms-"))
    resource = "/" + account + path
    for name in sorted(params, key=str.lower):
        resource += "\n%s:%s" % (name.lower(), params[name])
    string_to_sign = "\n".join(fields) + "\n" + canon_headers + resource
    sig = hmac.new(base64.b64decode(key_b64), string_to_sign.encode("utf-8"),
                   hashlib.sha256).digest()
    return "SharedKey %s:%s" % (account, base64.b64encode(sig).decode())


class AzureRemote(ObjectRemote):
    """Blob service REST API: Shared Key (``account`` + ``key``) or a SAS (``sas_url``)."""

    def __init__(self, conn: Connection):
        super().__init__(conn)
        cfg = conn.config
        self.account = cfg.get("account") or os.environ.get("AZURE_STORAGE_ACCOUNT", "")
        self.key = cfg.get("key") or os.environ.get("AZURE_STORAGE_KEY", "")
        self.sas: Dict[str, str] = {}
        endpoint = cfg.get("endpoint", "")
        if cfg.get("sas_url"):
            u = urllib.parse.urlsplit(cfg["sas_url"])
            self.sas = dict(urllib.parse.parse_qsl(u.query, keep_blank_values=True))
            endpoint = endpoint or "%s://%s" % (u.scheme, u.netloc)
            self.key = ""
        if not endpoint:
            if not self.account:
                raise ValueError("azureblob: no account (container_opts account/key or sas_url)")
            endpoint = "https://%s.blob.core.windows.net" % self.account
        if "://" not in endpoint:
            endpoint = "https://" + endpoint
        self.http = _Http(endpoint)
        self.prefix_path = self.http.base_path + "/" + _quote(self.bucket, "-_.~")

    def _request(self, method: str, key: Optional[str], params: Optional[Dict[str, str]] = None,
                 headers: Optional[Dict[str, str]] = None, body: bytes = b"",
                 ok: Tuple[int, ...] = (200, 201, 202, 204, 206)):
        path = self.prefix_path + ("/" + _quote(key) if key else "")
        params = dict(params or {})
        query = _query(dict(params, **self.sas))

        def sign() -> Dict[str, str]:
            h = dict(headers or {})
            h["x-ms-date"] = email.utils.formatdate(usegmt=True)
            h["x-ms-version"] = AZURE_VERSION
            h["Content-Length"] = str(len(body))
            if self.key:
                h["Authorization"] = azure_shared_key(self.account, self.key, method, path,
                                                      params, h)
            return h

        return self.http.request(method, path, query, sign, body, ok)

    def _head(self, key: str) -> Optional[int]:
        status, hdrs, _ = self._request("HEAD", key)
        return None if status == 404 else int(hdrs.get("content-length", "0"))

    def _list(self, prefix: str) -> Iterator[Tuple[str, int]]:
        marker = ""
        while True:
            params = {"restype": "container", "comp": "list", "prefix": prefix,
                      "maxresults": "5000"}
            if marker:
                params["marker"] = marker
            status, _, data = self._request("GET", None, params)
            if status == 404:
                raise ObjectStoreError("%s: no container %s" % (self, self.bucket))
            root = _xml_strip(ET.fromstring(data))
            for blob in root.iter("Blob"):
                yield blob.findtext("Name"), int(blob.findtext("Properties/Content-Length") or 0)
            marker = root.findtext("NextMarker") or ""
            if not marker:
                return

    def _put(self, key: str, data: bytes, meta: Dict[str, str]) -> None:
        headers = {"x-ms-blob-type": "BlockBlob", "Content-Type": "application/octet-stream",
                   "Content-MD5": base64.b64encode(hashlib.md5(data).digest()).decode()}
        headers.update({"x-ms-meta-" + k: v for k, v in meta.items()})
        self._request("PUT", key, headers=headers, body=data)

    def _get(self, key: str, start: int, end: int) -> bytes:
        status, _, data = self._request("GET", key,
                                        headers={"x-ms-range": "bytes=%d-%d" % (start, end)})
        if status == 404:
            raise FileNotFoundError("%s: no blob %s" % (self, key))
        return data

    def _upload_large(self, key, local, size, meta, pool) -> None:
        part = max(self.part, -(-size // 50000))  # a blob holds 50000 blocks
        nblocks = -(-size // part)
        ids = [base64.b64encode(b"tpi-%010d" % i).decode() for i in range(nblocks)]

        def send(index: int) -> None:
            offset = index * part
            with self._slots:
                body = self._read(local, offset, min(part, size - offset))
                self._request("PUT", key, {"comp": "block", "blockid": ids[index]},
                              {"Content-MD5": base64.b64encode(hashlib.md5(body).digest()).decode()},
                              body)

        for f in [pool.submit(send, i) for i in range(nblocks)]:
            f.result()
        body = ('<?xml version="1.0" encoding="utf-8"?><BlockList>%s</BlockList>' % "".join(
            "<Latest>%s</Latest>" % i for i in ids)).encode()
        headers = {"x-ms-blob-content-type": "application/octet-stream",
                   "Content-Type": "application/xml"}
        headers.update({"x-ms-meta-" + k: v for k, v in meta.items()})
        self._request("PUT", key, {"comp": "blocklist"}, headers, body)

    def _delete(self, keys: List[str]) -> None:
        def one(k: str) -> None:
            self._request("DELETE", k)  # a missing blob (404) is fine

        with ThreadPoolExecutor(self.threads) as pool:
            for f in [pool.submit(one, k) for k in keys]:
                f.result()


# -- Google Cloud Storage --------------------------------------------------------------------------

def _der(buf: bytes, i: int) -> Tuple[int, bytes, int]:
    """(tag, contents, next offset) of the DER element at ``i``."""
    tag = buf[i]
    length = buf[i + 1]
    i += 2
    if length & 0x80:
        n = length & 0x7F
        length = int.from_bytes(buf[i:i + n], "big")
        i += n
    return tag, buf[i:i + length], i + length


def _rsa_key(pem: str) -> Tuple[int, ...]:
    """(n, e, d, p, q, dp, dq, qinv) of a PEM RSA private key (PKCS#8 or PKCS#1)."""
    m = re.search(r"-----BEGIN ((?:RSA )?PRIVATE KEY)-----(.*?)-----END \1-----", pem, re.S)
    if not m:
        raise ValueError("no PEM private key")
    der = base64.b64decode("".join(m.group(2).split()))
    _, body, _ = _der(der, 0)
    if m.group(1) == "PRIVATE KEY":  # PKCS#8: version, algorithm, OCTET STRING(PKCS#1)
        i = 0
        _, _, i = _der(body, i)
        _, _, i = _der(body, i)
        tag, inner, _ = _der(body, i)
        if tag != 0x04:
            raise ValueError("not a PKCS#8 RSA key")
        _, body, _ = _der(inner, 0)
    ints, i = [], 0
    while i < len(body):
        tag, value, i = _der(body, i)
        if tag != 0x02:
            raise ValueError("malformed RSA key")
        ints.append(int.from_bytes(value, "big"))
    if len(ints) < 9:
        raise ValueError("malformed RSA key")
    return tuple(ints[1:9])


_SHA256_DIGEST_INFO = bytes.fromhex("3031300d060960864801650304020105000420")


def rs256_sign(pem: str, message: bytes) -> bytes:
    """RSASSA-PKCS1-v1_5 with SHA-256 (JWT ``RS256``), CRT exponentiation."""
    n, _e, _d, p, q, dp, dq, qinv = _rsa_key(pem)
    k = (n.bit_length() + 7) // 8
    t = _SHA256_DIGEST_INFO + hashlib.sha256(message).digest()
    em = b"\x00\x01" + b"\xff" * (k - len(t) - 3) + b"\x00" + t
    m = int.from_bytes(em, "big")
    s1, s2 = pow(m, dp, p), pow(m, dq, q)
    s = s2 + q * ((qinv * (s1 - s2)) % p)
    return s.to_bytes(k, "big")


def _range_end(headers: Dict[str, str]) -> int:
    """Last byte a GCS resumable session has kept, from a 308's ``Range: bytes=0-N`` (-1:
    no ``Range``, nothing kept yet)."""
    value = ""
    for k, v in (headers or {}).items():
        if k.lower() == "range":
            value = v
    m = re.match(r"^bytes=0-(\d+)$", value.strip())
    return int(m.group(1)) if m else -1


def _b64url(data: bytes) -> str:
    return base64.urlsafe_b64encode(data).rstrip(b"=").decode()


GCS_SCOPE = "https://www.googleapis.com/auth/devstorage.read_write"


class GCSRemote(ObjectRemote):
    """Cloud Storage JSON API with OAuth 2 bearer tokens (a service account's signed JWT
    exchanged at its ``token_uri``, or a given ``token``)."""

    def __init__(self, conn: Connection):
        super().__init__(conn)
        cfg = conn.config
        self.sa: Optional[Dict[str, str]] = None
        creds = cfg.get("service_account_credentials", "")
        path = cfg.get("service_account_file") or (
            "" if creds or cfg.get("token") else os.environ.get("GOOGLE_APPLICATION_CREDENTIALS", ""))
        if not creds and path:
            with open(os.path.expanduser(path)) as f:
                creds = f.read()
        if creds:
            self.sa = json.loads(creds)
        self._token = ""
        token = cfg.get("token", "")
        if token:
            try:  # rclone keeps an OAuth token as JSON
                token = json.loads(token).get("access_token", token)
            except (ValueError, AttributeError):
                pass
            self._token = token
        self._expiry = float("inf") if self._token else 0.0
        self._lock = threading.Lock()
        self.http = _Http(cfg.get("endpoint") or "https://storage.googleapis.com")
        self.obj_path = self.http.base_path + "/storage/v1/b/%s/o" % _quote(self.bucket, "-_.~")
        self.upload_path = self.http.base_path + "/upload/storage/v1/b/%s/o" % _quote(
            self.bucket, "-_.~")

    def _bearer(self) -> str:
        with self._lock:
            if self._token and time.time() < self._expiry - 60:
                return self._token
            if not self.sa:
                if self._token:
                    return self._token
                raise ObjectStoreError("googlecloudstorage: no credentials "
                                       "(service_account_credentials or token)")
            now = int(time.time())
            token_uri = self.sa.get("token_uri") or "https://oauth2.googleapis.com/token"
            header = _b64url(json.dumps({"alg": "RS256", "typ": "JWT"}).encode())
            claims = _b64url(json.dumps({"iss": self.sa["client_email"], "scope": GCS_SCOPE,
                                         "aud": token_uri, "iat": now,
                                         "exp": now + 3600}).encode())
            signing_input = ("%s.%s" % (header, claims)).encode()
            jwt = "%s.%s" % (signing_input.decode(),
                             _b64url(rs256_sign(self.sa["private_key"], signing_input)))
            body = urllib.parse.urlencode({
                "grant_type": "urn:ietf:params:oauth:grant-type:jwt-bearer",
                "assertion": jwt}).encode()
            tok = _Http(token_uri)
            status, _, data = tok.request(
                "POST", urllib.parse.urlsplit(token_uri).path or "/", "",
                lambda: {"Content-Type": "application/x-www-form-urlencoded"}, body)
            if status != 200:
                raise ObjectStoreError("token exchange at %s: HTTP %d" % (token_uri, status))
            reply = json.loads(data)
            self._token = reply["access_token"]
            self._expiry = time.time() + float(reply.get("expires_in", 3600))
            return self._token

    def _request(self, method: str, path: str, params: Optional[Dict[str, str]] = None,
                 headers: Optional[Dict[str, str]] = None, body: bytes = b"",
                 ok: Tuple[int, ...] = (200, 201, 204, 206)):
        query = _query(params or {})

        def sign() -> Dict[str, str]:
            h = dict(headers or {})
            h["Authorization"] = "Bearer " + self._bearer()
            return h

        return self.http.request(method, path, query, sign, body, ok)

    def _object(self, key: str) -> str:
        return self.obj_path + "/" + _quote(key, "-_.~")

    def _head(self, key: str) -> Optional[int]:
        status, _, data = self._request("GET", self._object(key), {"fields": "size"})
        return None if status == 404 else int(json.loads(data).get("size", 0))

    def _list(self, prefix: str) -> Iterator[Tuple[str, int]]:
        page = ""
        while True:
            params = {"prefix": prefix, "fields": "items(name,size),nextPageToken"}
            if page:
                params["pageToken"] = page
            status, _, data = self._request("GET", self.obj_path, params)
            if status == 404:
                raise ObjectStoreError("%s: no bucket %s" % (self, self.bucket))
            reply = json.loads(data)
            for item in reply.get("items", []):
                yield item["name"], int(item.get("size", 0))
            page = reply.get("nextPageToken", "")
            if not page:
                return

    def _put(self, key: str, data: bytes, meta: Dict[str, str]) -> None:
        """One request: a multipart upload, so the object gets its metadata (mtime) as on
        the S3 and Azure paths (``uploadType=media`` would drop it)."""
        boundary = "tpi-" + os.urandom(12).hex()
        head = json.dumps({"name": key, "metadata": meta}).encode()
        body = b"".join([
            b"--", boundary.encode(), b"\r\nContent-Type: application/json; charset=UTF-8\r\n\r\n",
            head, b"\r\n--", boundary.encode(),
            b"\r\nContent-Type: application/octet-stream\r\n\r\n", data,
            b"\r\n--", boundary.encode(), b"--\r\n"])
        self._request("POST", self.upload_path, {"uploadType": "multipart", "name": key},
                      {"Content-Type": "multipart/related; boundary=" + boundary}, body)

    def _get(self, key: str, start: int, end: int) -> bytes:
        status, _, data = self._request("GET", self._object(key), {"alt": "media"},
                                        {"Range": "bytes=%d-%d" % (start, end)})
        if status == 404:
            raise FileNotFoundError("%s: no object %s" % (self, key))
        return data

    def _upload_large(self, key, local, size, meta, pool) -> None:
        """One resumable session, parts in order (a session takes them sequentially)."""
        _, hdrs, _ = self._request(
            "POST", self.upload_path, {"uploadType": "resumable", "name": key},
            {"Content-Type": "application/json", "X-Upload-Content-Type":
             "application/octet-stream", "X-Upload-Content-Length": str(size)},
            json.dumps({"name": key, "metadata": meta}).encode())
        location = urllib.parse.urlsplit(hdrs["location"])
        path = location.path
        params = dict(urllib.parse.parse_qsl(location.query, keep_blank_values=True))
        part = max(256 << 10, self.part // (256 << 10) * (256 << 10))
        offset, stalls = 0, 0
        while offset < size:
            n = min(part, size - offset)
            with self._slots:
                body = self._read(local, offset, n)
                status, rh, _ = self._request(
                    "PUT", path, params,
                    {"Content-Range": "bytes %d-%d/%d" % (offset, offset + n - 1, size)}, body,
                    ok=(200, 201, 308))
            if status in (200, 201):
                if offset + n < size:
                    raise ObjectStoreError("%s: resumable upload of %s finished early at %d"
                                           % (self, key, offset + n))
                return
            # 308: the session kept bytes [0, N] -- possibly less than was sent (a retried or
            # cut-off PUT); resume from N + 1, never from where this loop thought it was
            got = _range_end(rh) + 1
            if got <= offset:
                stalls += 1
                if stalls > _Http.RETRIES:
                    raise ObjectStoreError("%s: resumable upload of %s stuck at %d" % (
                        self, key, got))
            else:
                stalls = 0
            if got > offset + n:
                raise ObjectStoreError("%s: resumable upload of %s: server kept %d bytes, "
                                       "%d were sent" % (self, key, got, offset + n))
            offset = got
        raise ObjectStoreError("%s: resumable upload of %s never completed" % (self, key))

    def _delete(self, keys: List[str]) -> None:
        def one(k: str) -> None:
            self._request("DELETE", self._object(k))

        with ThreadPoolExecutor(self.threads) as pool:
            for f in [pool.submit(one, k) for k in keys]:
                f.result()
