"""In-process fakes of the three object-store protocols of ``storage/objectstore.py``, served
from one threaded HTTP server on 127.0.0.1: S3 (path-style, Signature V4 checked), Azure Blob
(Azurite-style ``/<account>/<container>/<blob>``, Shared Key checked by a second, independent
implementation below) and Google Cloud Storage (JSON API; the service-account JWT is verified
with the ``openssl`` binary before a token is issued).

Every fake keeps its objects in memory, pages listings 3 entries at a time, honours ``Range``
and can be told to fail the next N requests with 503 (``fail_next``).
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import json
import os
import re
import subprocess
import tempfile
import threading
import urllib.parse
import uuid
import xml.etree.ElementTree as ET
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from terraform_provider_iterative_amd.storage.objectstore import sigv4_authorization

PAGE = 3
S3_ACCESS, S3_SECRET = "AKIDFAKE", "fake/secret+key"
AZ_ACCOUNT = "devacct"
AZ_KEY = base64.b64encode(b"azure-fake-key-0123456789abcdef").decode()
GCS_TOKEN = "ya29.fake-token"


class Store:
    def __init__(self):
        self.lock = threading.Lock()
        self.objects = {}     # (service, bucket) -> {key: bytes}
        self.meta = {}        # (service, bucket, key) -> {name: value}
        self.uploads = {}     # id -> {part/block id: bytes}
        self.fail_next = 0
        self.requests = []    # (service, method, path)
        self.auth_failures = 0
        self.missing_prefix = None  # writes into buckets with this name prefix: 404
        self.pubkey = None    # GCS: PEM of the service account's public key
        self.sa_email = ""
        self.gcs_short = []   # GCS resumable PUTs: keep this many bytes fewer of the next ones

    def bucket(self, service, name):
        return self.objects.setdefault((service, name), {})


def _azure_sign_independent(account, key_b64, method, raw_path, query, headers):
    """Shared Key as the Azure Storage REST documentation spells it out (kept apart from the
    client's code on purpose)."""
    h = {k.lower(): v for k, v in headers.items()}
    length = h.get("content-length", "")
    if length == "0":
        length = ""
    sts = method + "\n"
    for name in ("content-encoding", "content-language"):
        sts += h.get(name, "") + "\n"
    sts += length + "\n"
    for name in ("content-md5", "content-type", "date", "if-modified-since", "if-match",
                 "if-none-match", "if-unmodified-since", "range"):
        sts += h.get(name, "") + "\n"
    for name in sorted(k for k in h if k.startswith("x-ms-")):
        sts += "%s:%s\n" % (name, h[name].strip())
    sts += "/%s%s" % (account, raw_path)
    params = {}
    for k, v in urllib.parse.parse_qsl(query, keep_blank_values=True):
        params.setdefault(k.lower(), []).append(v)
    for k in sorted(params):
        sts += "\n%s:%s" % (k, ",".join(sorted(params[k])))
    digest = hmac.new(base64.b64decode(key_b64), sts.encode(), hashlib.sha256).digest()
    return "SharedKey %s:%s" % (account, base64.b64encode(digest).decode())


class Handler(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    store: Store = None

    def log_message(self, *args):
        pass

    # plumbing ---------------------------------------------------------------------------------
    def _body(self):
        n = int(self.headers.get("Content-Length") or 0)
        return self.rfile.read(n) if n else b""

    def _reply(self, status, body=b"", headers=None):
        self.send_response(status)
        for k, v in (headers or {}).items():
            self.send_header(k, v)
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        if self.command != "HEAD":
            self.wfile.write(body)

    def _range(self, data, header):
        m = re.match(r"bytes=(\d+)-(\d+)", header or "")
        if not m:
            return 200, data
        a, b = int(m.group(1)), int(m.group(2))
        return 206, data[a:b + 1]

    def _dispatch(self):
        body = self._body()
        u = urllib.parse.urlsplit(self.path)
        st = self.store
        with st.lock:
            st.requests.append((u.path.split("/")[1] if "/" in u.path else "", self.command,
                                u.path))
            if st.fail_next > 0:
                st.fail_next -= 1
                return self._reply(503, b"try again")
        if st.missing_prefix and self.command in ("PUT", "POST") and u.path != "/token" and \
                ("/" + st.missing_prefix) in u.path:
            return self._reply(404, b"<Error><Code>NoSuchBucket</Code></Error>")
        if u.path.startswith("/s3/"):
            return self._s3(u, body)
        if u.path.startswith("/" + AZ_ACCOUNT + "/"):
            return self._azure(u, body)
        if u.path == "/token":
            return self._token(body)
        if u.path.startswith("/storage/v1/") or u.path.startswith("/upload/storage/v1/"):
            return self._gcs(u, body)
        return self._reply(400, b"unknown service")

    do_GET = do_PUT = do_POST = do_DELETE = do_HEAD = _dispatch

    # S3 -----------------------------------------------------------------------------------------
    def _s3_auth(self, u, body):
        auth = self.headers.get("Authorization", "")
        m = re.match(r"AWS4-HMAC-SHA256 Credential=([^/]+)/(\d{8})/([^/]+)/s3/aws4_request,"
                     r"SignedHeaders=([^,]+),Signature=([0-9a-f]{64})$", auth)
        if not m or m.group(1) != S3_ACCESS:
            return False
        if self.headers.get("x-amz-content-sha256") != hashlib.sha256(body).hexdigest():
            return False
        signed = {n: self.headers.get(n, "") for n in m.group(4).split(";")}
        want = sigv4_authorization(self.command, u.path, u.query, signed,
                                   self.headers["x-amz-content-sha256"], m.group(3), "s3",
                                   S3_ACCESS, S3_SECRET, self.headers["x-amz-date"])
        return hmac.compare_digest(want, auth)

    def _s3(self, u, body):
        st = self.store
        if not self._s3_auth(u, body):
            with st.lock:
                st.auth_failures += 1
            return self._reply(403, b"<Error><Code>SignatureDoesNotMatch</Code></Error>")
        if self.headers.get("Content-MD5") and base64.b64encode(
                hashlib.md5(body).digest()).decode() != self.headers["Content-MD5"]:
            return self._reply(400, b"<Error><Code>BadDigest</Code></Error>")
        parts = u.path.split("/", 3)  # "", "s3", bucket, key
        bucket = urllib.parse.unquote(parts[2])
        key = urllib.parse.unquote(parts[3]) if len(parts) > 3 else ""
        q = dict(urllib.parse.parse_qsl(u.query, keep_blank_values=True))
        with st.lock:
            objs = st.bucket("s3", bucket)
            if not key and self.command == "GET":
                names = sorted(k for k in objs if k.startswith(q.get("prefix", "")))
                start = int(q.get("continuation-token") or 0)
                page = names[start:start + PAGE]
                more = start + PAGE < len(names)
                xml = "".join("<Contents><Key>%s</Key><Size>%d</Size></Contents>"
                              % (k.replace("&", "&amp;").replace("<", "&lt;"), len(objs[k]))
                              for k in page)
                doc = ('<ListBucketResult xmlns="http://s3.amazonaws.com/doc/2006-03-01/">%s'
                       '<IsTruncated>%s</IsTruncated>%s</ListBucketResult>' % (
                           xml, "true" if more else "false",
                           "<NextContinuationToken>%d</NextContinuationToken>" % (start + PAGE)
                           if more else ""))
                return self._reply(200, doc.encode())
            if not key and self.command == "POST" and "delete" in q:
                root = ET.fromstring(body)
                for k in root.iter("Key"):
                    objs.pop(k.text, None)
                return self._reply(200, b"<DeleteResult/>")
            if self.command == "POST" and "uploads" in q:
                uid = uuid.uuid4().hex
                st.uploads[uid] = {}
                st.meta[("s3", bucket, key)] = {k: v for k, v in self.headers.items()
                                                if k.lower().startswith("x-amz-meta-")}
                return self._reply(200, ("<InitiateMultipartUploadResult><UploadId>%s"
                                         "</UploadId></InitiateMultipartUploadResult>"
                                         % uid).encode())
            if self.command == "PUT" and "uploadId" in q:
                st.uploads[q["uploadId"]][int(q["partNumber"])] = body
                return self._reply(200, headers={"ETag": '"%s"' % hashlib.md5(body).hexdigest()})
            if self.command == "POST" and "uploadId" in q:
                parts_ = st.uploads.pop(q["uploadId"])
                root = ET.fromstring(body)
                data = b""
                for p in root.iter("Part"):
                    n = int(p.findtext("PartNumber"))
                    if p.findtext("ETag") != '"%s"' % hashlib.md5(parts_[n]).hexdigest():
                        return self._reply(200, b"<Error><Code>InvalidPart</Code>"
                                                b"<Message>etag</Message></Error>")
                    data += parts_[n]
                objs[key] = data
                return self._reply(200, b"<CompleteMultipartUploadResult/>")
            if self.command == "DELETE" and "uploadId" in q:
                st.uploads.pop(q["uploadId"], None)
                return self._reply(204)
            if self.command == "PUT":
                objs[key] = body
                st.meta[("s3", bucket, key)] = {k: v for k, v in self.headers.items()
                                                if k.lower().startswith("x-amz-meta-")}
                return self._reply(200, headers={"ETag": '"%s"' % hashlib.md5(body).hexdigest()})
            if key not in objs:
                return self._reply(404, b"<Error><Code>NoSuchKey</Code></Error>")
            if self.command == "HEAD":
                self.send_response(200)
                self.send_header("Content-Length", str(len(objs[key])))
                self.end_headers()
                return None
            if self.command == "GET":
                status, data = self._range(objs[key], self.headers.get("Range"))
                return self._reply(status, data)
            if self.command == "DELETE":
                objs.pop(key, None)
                return self._reply(204)
        return self._reply(400)

    # Azure --------------------------------------------------------------------------------------
    def _azure(self, u, body):
        st = self.store
        want = _azure_sign_independent(AZ_ACCOUNT, AZ_KEY, self.command, u.path, u.query,
                                       dict(self.headers.items()))
        if self.headers.get("Authorization") != want:
            with st.lock:
                st.auth_failures += 1
            return self._reply(403, b"<Error><Code>AuthenticationFailed</Code></Error>")
        parts = u.path.split("/", 3)  # "", account, container, blob
        container = urllib.parse.unquote(parts[2])
        blob = urllib.parse.unquote(parts[3]) if len(parts) > 3 else ""
        q = dict(urllib.parse.parse_qsl(u.query, keep_blank_values=True))
        with st.lock:
            objs = st.bucket("az", container)
            if not blob and q.get("comp") == "list":
                names = sorted(k for k in objs if k.startswith(q.get("prefix", "")))
                start = int(q.get("marker") or 0)
                page = names[start:start + PAGE]
                nxt = str(start + PAGE) if start + PAGE < len(names) else ""
                xml = "".join("<Blob><Name>%s</Name><Properties><Content-Length>%d"
                              "</Content-Length></Properties></Blob>"
                              % (k.replace("&", "&amp;").replace("<", "&lt;"), len(objs[k]))
                              for k in page)
                return self._reply(200, ("<EnumerationResults><Blobs>%s</Blobs><NextMarker>%s"
                                         "</NextMarker></EnumerationResults>" % (xml, nxt)
                                         ).encode())
            if self.command == "PUT" and q.get("comp") == "block":
                st.uploads.setdefault((container, blob), {})[q["blockid"]] = body
                return self._reply(201)
            if self.command == "PUT" and q.get("comp") == "blocklist":
                blocks = st.uploads.pop((container, blob), {})
                root = ET.fromstring(body)
                objs[blob] = b"".join(blocks[e.text] for e in root.iter("Latest"))
                return self._reply(201)
            if self.command == "PUT":
                if self.headers.get("x-ms-blob-type") != "BlockBlob":
                    return self._reply(400)
                objs[blob] = body
                st.meta[("az", container, blob)] = {k: v for k, v in self.headers.items()
                                                    if k.lower().startswith("x-ms-meta-")}
                return self._reply(201)
            if blob not in objs:
                return self._reply(404, b"<Error><Code>BlobNotFound</Code></Error>")
            if self.command == "HEAD":
                self.send_response(200)
                self.send_header("Content-Length", str(len(objs[blob])))
                self.end_headers()
                return None
            if self.command == "GET":
                status, data = self._range(objs[blob], self.headers.get("x-ms-range"))
                return self._reply(status, data)
            if self.command == "DELETE":
                objs.pop(blob, None)
                return self._reply(202)
        return self._reply(400)

    # GCS ----------------------------------------------------------------------------------------
    def _token(self, body):
        st = self.store
        form = dict(urllib.parse.parse_qsl(body.decode()))
        jwt = form.get("assertion", "")
        try:
            head, claims, sig = jwt.split(".")
            pad = lambda s: base64.urlsafe_b64decode(s + "=" * (-len(s) % 4))  # noqa: E731
            claims_doc = json.loads(pad(claims))
            with tempfile.TemporaryDirectory() as d:
                for name, data in (("pub.pem", st.pubkey.encode()), ("sig", pad(sig)),
                                   ("msg", ("%s.%s" % (head, claims)).encode())):
                    with open(os.path.join(d, name), "wb") as f:
                        f.write(data)
                ok = subprocess.run(["openssl", "dgst", "-sha256", "-verify",
                                     os.path.join(d, "pub.pem"), "-signature",
                                     os.path.join(d, "sig"), os.path.join(d, "msg")],
                                    capture_output=True).returncode == 0
        except Exception:
            ok = False
        if not ok or claims_doc.get("iss") != st.sa_email or \
                form.get("grant_type") != "urn:ietf:params:oauth:grant-type:jwt-bearer":
            with st.lock:
                st.auth_failures += 1
            return self._reply(400, b'{"error": "invalid_grant"}')
        return self._reply(200, json.dumps({"access_token": GCS_TOKEN, "expires_in": 3600,
                                            "token_type": "Bearer"}).encode())

    def _gcs(self, u, body):
        st = self.store
        if self.headers.get("Authorization") != "Bearer " + GCS_TOKEN:
            with st.lock:
                st.auth_failures += 1
            return self._reply(401, b'{"error": "unauthorized"}')
        q = dict(urllib.parse.parse_qsl(u.query, keep_blank_values=True))
        m = re.match(r"^(/upload)?/storage/v1/b/([^/]+)/o(?:/(.+))?$", u.path)
        if not m:
            return self._reply(400)
        upload, bucket = bool(m.group(1)), urllib.parse.unquote(m.group(2))
        name = urllib.parse.unquote(m.group(3)) if m.group(3) else ""
        with st.lock:
            objs = st.bucket("gs", bucket)
            if upload and q.get("uploadType") == "media":
                objs[q["name"]] = body
                return self._reply(200, json.dumps({"name": q["name"]}).encode())
            if upload and q.get("uploadType") == "multipart":
                ctype = self.headers.get("Content-Type", "")
                bm = re.match(r"multipart/related; boundary=(\S+)$", ctype)
                if not bm:
                    return self._reply(400, b"not multipart/related")
                sep = b"--" + bm.group(1).encode()
                parts = [p for p in body.split(sep)[1:] if not p.startswith(b"--")]
                if len(parts) != 2:
                    return self._reply(400, b"expected metadata + media")
                docs = []
                for part in parts:
                    head, _, payload = part.partition(b"\r\n\r\n")
                    docs.append(payload[:-2] if payload.endswith(b"\r\n") else payload)
                meta = json.loads(docs[0])
                objs[meta["name"]] = docs[1]
                st.meta[("gs", bucket, meta["name"])] = dict(meta.get("metadata") or {})
                return self._reply(200, json.dumps({"name": meta["name"]}).encode())
            if upload and q.get("uploadType") == "resumable" and self.command == "POST":
                uid = uuid.uuid4().hex
                st.uploads[uid] = {"name": q["name"], "data": b"",
                                   "size": int(self.headers["X-Upload-Content-Length"]),
                                   "metadata": dict(json.loads(body or b"{}").get("metadata")
                                                    or {})}
                loc = "http://%s:%d/upload/storage/v1/b/%s/o?uploadType=resumable&upload_id=%s" % (
                    self.server.server_address[0], self.server.server_address[1],
                    urllib.parse.quote(bucket), uid)
                return self._reply(200, headers={"Location": loc})
            if upload and self.command == "PUT":
                up = st.uploads[q["upload_id"]]
                r = re.match(r"bytes (\d+)-(\d+)/(\d+)", self.headers["Content-Range"])
                a, b, total = int(r.group(1)), int(r.group(2)), int(r.group(3))
                if a != len(up["data"]) or total != up["size"] or b - a + 1 != len(body):
                    return self._reply(400, b"bad range")
                if st.gcs_short:  # the session keeps only part of this chunk
                    body = body[:max(0, len(body) - st.gcs_short.pop(0))]
                up["data"] += body
                if len(up["data"]) < total:
                    kept = len(up["data"])
                    return self._reply(308, headers={"Range": "bytes=0-%d" % (kept - 1)}
                                       if kept else {})
                objs[up["name"]] = up["data"]
                st.meta[("gs", bucket, up["name"])] = up["metadata"]
                del st.uploads[q["upload_id"]]
                return self._reply(200, json.dumps({"name": up["name"]}).encode())
            if not name and self.command == "GET":
                names = sorted(k for k in objs if k.startswith(q.get("prefix", "")))
                start = int(q.get("pageToken") or 0)
                page = names[start:start + PAGE]
                doc = {"items": [{"name": k, "size": str(len(objs[k]))} for k in page]}
                if start + PAGE < len(names):
                    doc["nextPageToken"] = str(start + PAGE)
                return self._reply(200, json.dumps(doc).encode())
            if name not in objs:
                return self._reply(404, b'{"error": "not found"}')
            if self.command == "GET" and q.get("alt") == "media":
                status, data = self._range(objs[name], self.headers.get("Range"))
                return self._reply(status, data)
            if self.command == "GET":
                return self._reply(200, json.dumps({"name": name,
                                                    "size": str(len(objs[name]))}).encode())
            if self.command == "DELETE":
                objs.pop(name, None)
                return self._reply(204)
        return self._reply(400)


class FakeObjectStores:
    """``with FakeObjectStores(tmpdir) as fake:`` -- ``fake.endpoint``, ``fake.store`` and
    ``fake.gcs_credentials`` (service-account JSON whose key was made by ``openssl``)."""

    def __init__(self, tmpdir):
        self.store = Store()
        key = os.path.join(str(tmpdir), "sa.pem")
        subprocess.run(["openssl", "genpkey", "-algorithm", "RSA", "-pkeyopt",
                        "rsa_keygen_bits:2048", "-out", key], check=True, capture_output=True)
        self.store.pubkey = subprocess.run(["openssl", "pkey", "-in", key, "-pubout"],
                                           check=True, capture_output=True).stdout.decode()
        self.store.sa_email = "tpi-test@example.iam.gserviceaccount.com"
        self.private_key = open(key).read()
        handler = type("H", (Handler,), {"store": self.store})
        self.server = ThreadingHTTPServer(("127.0.0.1", 0), handler)
        self.server.daemon_threads = True
        self.endpoint = "http://127.0.0.1:%d" % self.server.server_address[1]
        self.thread = threading.Thread(target=self.server.serve_forever, daemon=True)

    @property
    def gcs_credentials(self) -> str:
        return json.dumps({"type": "service_account", "client_email": self.store.sa_email,
                           "private_key": self.private_key,
                           "token_uri": self.endpoint + "/token"})

    def options(self, backend: str) -> dict:
        """``container_opts`` that point a connection of ``backend`` at this fake."""
        if backend == "s3":
            return {"endpoint": self.endpoint + "/s3", "access_key_id": S3_ACCESS,
                    "secret_access_key": S3_SECRET, "region": "us-east-1"}
        if backend == "azureblob":
            return {"endpoint": self.endpoint + "/" + AZ_ACCOUNT, "account": AZ_ACCOUNT,
                    "key": AZ_KEY}
        return {"endpoint": self.endpoint, "service_account_credentials": self.gcs_credentials}

    def objects(self, backend: str, bucket: str) -> dict:
        service = {"s3": "s3", "azureblob": "az", "googlecloudstorage": "gs"}[backend]
        return self.store.bucket(service, bucket)

    def __enter__(self):
        self.thread.start()
        return self

    def __exit__(self, *exc):
        self.server.shutdown()
        self.server.server_close()
