"""Terraform plugin server: go-plugin handshake + tfplugin5 gRPC service.

``terraform-provider-iterative`` (``bin/``) runs :func:`serve`, making this framework a
drop-in provider binary for a real ``terraform`` (reference: ``main.go:11-18`` serving
``iterative.Provider()``):

* handshake: checks ``TF_PLUGIN_MAGIC_COOKIE``, negotiates protocol 5 from
  ``PLUGIN_PROTOCOL_VERSIONS``, listens on a Unix socket and prints
  ``1|5|unix|<path>|grpc|<cert>``; with AutoMTLS (``PLUGIN_CLIENT_CERT``) it serves TLS with a
  fresh self-signed certificate and requires Terraform's client certificate;
* services: ``tfplugin5.Provider`` (schema, validate, plan, apply, read, import, upgrade),
  ``grpc.health.v1.Health`` and go-plugin's ``GRPCController``/``GRPCStdio``/``GRPCBroker``.

Plan/apply follow terraform-plugin-sdk v2 semantics (defaults in the plan, unknown computed
values on create, ``requires_replace`` for ForceNew, ``legacy_type_system``).
"""
from __future__ import annotations

import base64
import json
import os
import subprocess
import sys
import tempfile
import threading
from concurrent import futures
from typing import Any, Dict, Optional, Tuple

import grpc

from ..models.schema import (SCHEMAS, SchemaError, force_new_changes, get_schema, normalize)
from . import cty, resources
from . import tfplugin5 as pb

MAGIC_COOKIE_KEY = "TF_PLUGIN_MAGIC_COOKIE"
MAGIC_COOKIE_VALUE = "d602bf8f470bc67ca7faa0386276bbdd4330efaf76d1a219cb4d6991ca9872b2"
CORE_PROTOCOL_VERSION = 1
APP_PROTOCOL_VERSION = 5


# ---- schema -------------------------------------------------------------------------------------

def _schema_message(schema) -> Any:
    msg = pb.Schema()
    msg.version = schema.version
    block = msg.block
    block.version = schema.version
    id_attr = block.attributes.add()
    id_attr.name, id_attr.type, id_attr.optional, id_attr.computed = "id", b'"string"', True, True
    for name, attr in sorted(schema.attributes.items()):
        if attr.is_block:
            nb = block.block_types.add()
            nb.type_name = name
            nb.nesting = 3  # SET
            for k, a in sorted(attr.elem.items()):
                sub = nb.block.attributes.add()
                sub.name = k
                sub.type = json.dumps(cty.type_json(cty._attr_type(a))).encode()
                sub.optional, sub.required, sub.computed = a.optional, a.required, a.computed
                sub.sensitive = a.sensitive
            continue
        a = block.attributes.add()
        a.name = name
        a.type = json.dumps(cty.type_json(cty._attr_type(attr))).encode()
        a.required = attr.required
        a.optional = attr.optional
        a.computed = attr.computed  # defaults are applied in the plan, as SDKv2 does
        a.sensitive = attr.sensitive
    if schema.timeouts:
        nb = block.block_types.add()
        nb.type_name = "timeouts"
        nb.nesting = 1  # SINGLE
        for k in cty.TIMEOUT_KEYS:
            if k in schema.timeouts:
                sub = nb.block.attributes.add()
                sub.name, sub.type, sub.optional = k, b'"string"', True
    return msg


def _diag(severity: str, summary: str, detail: str = ""):
    d = pb.Diagnostic()
    d.severity = 1 if severity == "error" else 2
    d.summary = summary
    d.detail = detail
    return d


def _dv(value: Any, t) -> Any:
    v = pb.DynamicValue()
    v.msgpack = cty.encode_msgpack(value, t)
    return v


def _read_dv(dv, t) -> Any:
    if dv is None:
        return None
    if dv.msgpack:
        return cty.decode_msgpack(dv.msgpack)
    if dv.json:
        return cty.decode_json(dv.json, t)
    return None


# ---- the provider service -----------------------------------------------------------------------

class ProviderService:
    def __init__(self, stop_event: threading.Event):
        self.stop_event = stop_event

    def _schema(self, type_name: str):
        return get_schema(type_name)

    def GetSchema(self, request, context):
        _, Res = pb.classes("GetSchema")
        res = Res()
        res.provider.block.version = 0
        for name, schema in SCHEMAS.items():
            res.resource_schemas[name].CopyFrom(_schema_message(schema))
        res.server_capabilities.plan_destroy = False
        return res

    def PrepareProviderConfig(self, request, context):
        _, Res = pb.classes("PrepareProviderConfig")
        res = Res()
        res.prepared_config.CopyFrom(request.config)
        return res

    def Configure(self, request, context):
        return pb.classes("Configure")[1]()

    def ValidateResourceTypeConfig(self, request, context):
        _, Res = pb.classes("ValidateResourceTypeConfig")
        res = Res()
        try:
            schema = self._schema(request.type_name)
            value = _read_dv(request.config, cty.block_type(schema))
            attrs, _ = cty.from_wire(value, schema)
            attrs = {k: v for k, v in attrs.items() if v is not None and k != "id"}
            _validate_known(request.type_name, attrs)
        except SchemaError as error:
            res.diagnostics.append(_diag("error", str(error)))
        return res

    def ValidateDataSourceConfig(self, request, context):
        _, Res = pb.classes("ValidateDataSourceConfig")
        res = Res()
        res.diagnostics.append(_diag("error", "unknown data source %s" % request.type_name))
        return res

    def UpgradeResourceState(self, request, context):
        _, Res = pb.classes("UpgradeResourceState")
        res = Res()
        schema = self._schema(request.type_name)
        t = cty.block_type(schema)
        raw = request.raw_state.json
        if raw:
            value = cty.decode_json(raw, t)
        else:  # legacy flatmap states are not produced by this provider
            value = None
        res.upgraded_state.CopyFrom(_dv(value, t))
        return res

    def ReadResource(self, request, context):
        _, Res = pb.classes("ReadResource")
        res = Res()
        schema = self._schema(request.type_name)
        t = cty.block_type(schema)
        current = _read_dv(request.current_state, t)
        res.private = request.private
        if current is None:
            res.new_state.CopyFrom(_dv(None, t))
            return res
        attrs, timeouts = cty.from_wire(current, schema)
        result = resources.handler(request.type_name, "read")(attrs, timeouts)
        for d in result.diagnostics:
            res.diagnostics.append(_diag(d.severity, d.summary, d.detail))
        state = result.state if result.id else None
        res.new_state.CopyFrom(_dv(cty.to_wire(state, schema, current.get("timeouts"))
                                   if state else None, t))
        return res

    def PlanResourceChange(self, request, context):
        _, Res = pb.classes("PlanResourceChange")
        res = Res()
        res.legacy_type_system = True
        schema = self._schema(request.type_name)
        t = cty.block_type(schema)
        prior = _read_dv(request.prior_state, t)
        proposed = _read_dv(request.proposed_new_state, t)
        res.planned_private = request.prior_private
        if proposed is None:  # destroy
            res.planned_state.CopyFrom(_dv(None, t))
            return res
        planned = dict(proposed)
        # defaults for unset optional attributes (SDKv2 puts Default into the plan)
        for name, attr in schema.attributes.items():
            if attr.is_block:
                blocks = []
                for b in planned.get(name) or []:
                    nb = dict(b)
                    for k, a in attr.elem.items():
                        if nb.get(k) is None and a.default is not None:
                            nb[k] = a.default
                    blocks.append(nb)
                planned[name] = blocks
            elif planned.get(name) is None and attr.default is not None and \
                    (attr.optional or attr.required):
                planned[name] = attr.default
        computed = [n for n, a in schema.attributes.items()
                    if a.computed and not a.optional and not a.required]
        if prior is None:
            planned["id"] = cty.UNKNOWN
            for name in computed:
                planned[name] = cty.UNKNOWN
        else:
            planned["id"] = prior.get("id")
            old, _ = cty.from_wire(prior, schema)
            new, _ = cty.from_wire(planned, schema)
            replace = force_new_changes(request.type_name, old, new)
            if replace:
                planned["id"] = cty.UNKNOWN
                for name in computed:
                    planned[name] = cty.UNKNOWN
                for path in sorted({r.split(".")[0] for r in replace}):
                    step = res.requires_replace.add().steps.add()
                    step.attribute_name = path
            else:
                for name in computed:
                    planned[name] = prior.get(name)
        res.planned_state.CopyFrom(_dv(planned, t))
        return res

    def ApplyResourceChange(self, request, context):
        _, Res = pb.classes("ApplyResourceChange")
        res = Res()
        res.legacy_type_system = True
        schema = self._schema(request.type_name)
        t = cty.block_type(schema)
        prior = _read_dv(request.prior_state, t)
        planned = _read_dv(request.planned_state, t)
        if planned is None:  # delete
            attrs, timeouts = cty.from_wire(prior, schema)
            result = resources.handler(request.type_name, "delete")(attrs, timeouts)
            for d in result.diagnostics:
                res.diagnostics.append(_diag(d.severity, d.summary, d.detail))
            res.new_state.CopyFrom(_dv(prior if not result.ok else None, t))
            return res
        attrs, timeouts = cty.from_wire(planned, schema)
        try:
            attrs = _normalize_keep(request.type_name, attrs)
        except SchemaError as error:
            res.diagnostics.append(_diag("error", str(error)))
            res.new_state.CopyFrom(_dv(prior, t))
            return res
        op = "create" if prior is None else "read"
        if prior is not None:
            attrs["id"] = prior.get("id")
            for name, attr in schema.attributes.items():
                if attr.computed and attrs.get(name) is None:
                    attrs[name] = prior.get(name)
        result = resources.handler(request.type_name, op)(attrs, timeouts)
        for d in result.diagnostics:
            res.diagnostics.append(_diag(d.severity, d.summary, d.detail))
        if not result.id:
            res.new_state.CopyFrom(_dv(prior, t) if prior is not None else _dv(None, t))
            return res
        state = dict(result.state)
        state["id"] = result.id
        res.new_state.CopyFrom(_dv(cty.to_wire(state, schema, planned.get("timeouts")), t))
        res.private = base64.b64decode(_private(timeouts))
        return res

    def ImportResourceState(self, request, context):
        _, Res = pb.classes("ImportResourceState")
        res = Res()
        schema = self._schema(request.type_name)
        t = cty.block_type(schema)
        attrs = _import_attrs(request.type_name, request.id)
        if attrs is None:
            res.diagnostics.append(_diag("error", "cannot import %s %r: not found on this node"
                                         % (request.type_name, request.id)))
            return res
        imported = res.imported_resources.add()
        imported.type_name = request.type_name
        imported.state.CopyFrom(_dv(cty.to_wire(attrs, schema), t))
        return res

    def ReadDataSource(self, request, context):
        _, Res = pb.classes("ReadDataSource")
        res = Res()
        res.diagnostics.append(_diag("error", "unknown data source %s" % request.type_name))
        return res

    def Stop(self, request, context):
        return pb.classes("Stop")[1]()


def _private(timeouts: Dict[str, float]) -> str:
    from .state import encode_private

    return encode_private(timeouts)


def _validate_known(type_name: str, attrs: Dict[str, Any]) -> None:
    schema = get_schema(type_name)
    unknown = set(attrs) - set(schema.attributes) - {"timeouts"}
    if unknown:
        raise SchemaError("%s: unsupported argument(s): %s" % (type_name, ", ".join(sorted(unknown))))


def _normalize_keep(type_name: str, attrs: Dict[str, Any]) -> Dict[str, Any]:
    """normalize() but keep computed values that are already set."""
    schema = get_schema(type_name)
    config = {k: v for k, v in attrs.items() if k in schema.attributes and
              not (schema.attributes[k].computed and not schema.attributes[k].optional
                   and not schema.attributes[k].required)}
    out = normalize(type_name, config)
    for k, v in attrs.items():
        if k not in config:
            out[k] = v
    return out


def _import_attrs(type_name: str, rid: str) -> Optional[Dict[str, Any]]:
    from ..models.cloud import default_state_root

    root = default_state_root()
    for provider in ("mi355x", "local"):
        path = os.path.join(root, provider, rid, "task.json")
        if os.path.exists(path):
            with open(path) as handle:
                d = json.load(handle)
            script = ""
            spath = os.path.join(root, provider, rid, "supervisor", "script")
            if os.path.exists(spath):
                with open(spath) as handle:
                    script = handle.read()
            attrs = normalize("iterative_task", {
                "cloud": provider, "region": d.get("region") or "us-west",
                "machine": d.get("machine") or "m", "script": script or "#!/bin/sh\n",
                "parallelism": d.get("parallelism", 1), "spot": d.get("spot", -1),
                "timeout": int(d.get("timeout") or 86400), "tags": d.get("tags") or None})
            attrs["id"] = rid
            return attrs if type_name == "iterative_task" else None
    return None


# ---- go-plugin plumbing ----------------------------------------------------------------------------

def _health_handler():
    def check(request, context):
        return b"\x08\x01"  # HealthCheckResponse{status: SERVING}

    return grpc.method_handlers_generic_handler("grpc.health.v1.Health", {
        "Check": grpc.unary_unary_rpc_method_handler(check, request_deserializer=lambda b: b,
                                                     response_serializer=lambda b: b)})


def _controller_handlers(stop_event: threading.Event):
    def shutdown(request, context):
        stop_event.set()
        return b""

    def stdio(request, context):
        stop_event.wait()
        return iter(())

    def broker(request_iterator, context):
        for _ in request_iterator:
            pass
        return iter(())

    ident = dict(request_deserializer=lambda b: b, response_serializer=lambda b: b)
    return [
        grpc.method_handlers_generic_handler("plugin.GRPCController", {
            "Shutdown": grpc.unary_unary_rpc_method_handler(shutdown, **ident)}),
        grpc.method_handlers_generic_handler("plugin.GRPCStdio", {
            "StreamStdio": grpc.unary_stream_rpc_method_handler(stdio, **ident)}),
        grpc.method_handlers_generic_handler("plugin.GRPCBroker", {
            "StartStream": grpc.stream_stream_rpc_method_handler(broker, **ident)}),
    ]


def provider_handler(service: ProviderService):
    handlers = {}
    for method in pb.METHODS:
        Req, Res = pb.classes(method)
        handlers[method] = grpc.unary_unary_rpc_method_handler(
            getattr(service, method), request_deserializer=Req.FromString,
            response_serializer=Res.SerializeToString)
    return grpc.method_handlers_generic_handler(pb.SERVICE, handlers)


def make_server(max_workers: int = 16) -> Tuple[grpc.Server, threading.Event]:
    stop = threading.Event()
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers))
    server.add_generic_rpc_handlers([provider_handler(ProviderService(stop)), _health_handler(),
                                     *_controller_handlers(stop)])
    return server, stop


def generate_cert(directory: str) -> Tuple[bytes, bytes]:
    """Self-signed localhost certificate (go-plugin AutoMTLS server side)."""
    key, cert = os.path.join(directory, "key.pem"), os.path.join(directory, "cert.pem")
    subprocess.run(["openssl", "req", "-x509", "-newkey", "ec", "-pkeyopt",
                    "ec_paramgen_curve:P-256", "-nodes", "-keyout", key, "-out", cert, "-days",
                    "30", "-subj", "/O=HashiCorp/CN=localhost", "-addext",
                    "subjectAltName=DNS:localhost", "-addext",
                    "basicConstraints=critical,CA:TRUE", "-addext",
                    "keyUsage=digitalSignature,keyEncipherment,keyAgreement,keyCertSign"],
                   check=True, capture_output=True)
    with open(key, "rb") as k, open(cert, "rb") as c:
        return k.read(), c.read()


def _der_b64(cert_pem: bytes) -> str:
    body = b"".join(l for l in cert_pem.splitlines() if not l.startswith(b"-----"))
    return base64.b64encode(base64.b64decode(body)).decode().rstrip("=")


def serve(environ=None, out=None) -> int:
    environ = os.environ if environ is None else environ
    out = out or sys.stdout
    if "--version" in sys.argv[1:]:
        from .._version import __version__

        out.write("terraform-provider-iterative v%s\n" % __version__)
        return 0
    if environ.get(MAGIC_COOKIE_KEY) != MAGIC_COOKIE_VALUE:
        sys.stderr.write("This binary is a plugin. These are not meant to be executed directly.\n"
                         "Please execute the program that consumes these plugins, which will\n"
                         "load any plugins automatically\n")
        return 1
    versions = [v.strip() for v in environ.get("PLUGIN_PROTOCOL_VERSIONS", "5").split(",")]
    if str(APP_PROTOCOL_VERSION) not in versions:
        sys.stderr.write("Incompatible API version with plugin. Plugin version: 5, Client "
                         "versions: %s\n" % ",".join(versions))
        return 1
    server, stop = make_server()
    tmp = tempfile.mkdtemp(prefix="plugin")
    sock = os.path.join(tmp, "plugin.sock")
    client_cert = environ.get("PLUGIN_CLIENT_CERT")
    cert_field = ""
    if client_cert:
        key, cert = generate_cert(tmp)
        creds = grpc.ssl_server_credentials([(key, cert)], root_certificates=client_cert.encode(),
                                            require_client_auth=True)
        server.add_secure_port("unix:" + sock, creds)
        cert_field = _der_b64(cert)
    else:
        server.add_insecure_port("unix:" + sock)
    server.start()
    out.write("%d|%d|unix|%s|grpc|%s\n" % (CORE_PROTOCOL_VERSION, APP_PROTOCOL_VERSION, sock,
                                           cert_field))
    out.flush()
    try:
        stop.wait()
    except KeyboardInterrupt:  # pragma: no cover
        pass
    server.stop(grace=2)
    from ..utils import analytics

    analytics.wait_for_analytics()
    return 0
