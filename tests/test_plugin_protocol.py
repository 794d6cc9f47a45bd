"""tfplugin5 server: handshake (with AutoMTLS) and the plan/apply/read/destroy lifecycle as
Terraform core would drive it over gRPC."""
import base64
import json
import os
import subprocess
import sys
import time

import grpc
import pytest

from terraform_provider_iterative_amd.provider import cty
from terraform_provider_iterative_amd.provider import tfplugin5 as pb
from terraform_provider_iterative_amd.provider.server import (MAGIC_COOKIE_KEY,
                                                              MAGIC_COOKIE_VALUE, make_server)
from terraform_provider_iterative_amd.models.schema import get_schema

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class Client:
    def __init__(self, channel):
        self.channel = channel

    def call(self, method, request):
        Req, Res = pb.classes(method)
        fn = self.channel.unary_unary("/tfplugin5.Provider/" + method,
                                      request_serializer=Req.SerializeToString,
                                      response_deserializer=Res.FromString)
        return fn(request, timeout=120)

    def req(self, method):
        return pb.classes(method)[0]()


@pytest.fixture()
def client(tmp_path, monkeypatch):
    monkeypatch.setenv("TPI_STATE_ROOT", str(tmp_path / "state"))
    server, stop = make_server()
    sock = str(tmp_path / "p.sock")
    server.add_insecure_port("unix:" + sock)
    server.start()
    channel = grpc.insecure_channel("unix:" + sock)
    yield Client(channel)
    channel.close()
    server.stop(0)


def dv(value, t):
    d = pb.DynamicValue()
    d.msgpack = cty.encode_msgpack(value, t)
    return d


def test_schema(client):
    res = client.call("GetSchema", client.req("GetSchema"))
    assert set(res.resource_schemas) == {"iterative_task", "iterative_machine",
                                         "iterative_cml_runner"}
    task = res.resource_schemas["iterative_task"].block
    attrs = {a.name: a for a in task.attributes}
    assert attrs["cloud"].required and attrs["script"].required
    assert json.loads(attrs["status"].type) == ["map", "number"] and attrs["status"].computed
    assert attrs["ssh_private_key"].sensitive and attrs["id"].computed
    blocks = {b.type_name: b for b in task.block_types}
    assert blocks["storage"].nesting == 3 and blocks["timeouts"].nesting == 1


def test_lifecycle(client, tmp_path):
    schema = get_schema("iterative_task")
    t = cty.block_type(schema)
    config = {k: None for k in t[1]}
    config.update({"cloud": "local", "machine": "s", "name": "plugin-test",
                   "script": "#!/bin/sh\necho from-plugin\n", "storage": []})
    # validate
    req = client.req("ValidateResourceTypeConfig")
    req.type_name = "iterative_task"
    req.config.CopyFrom(dv(config, t))
    assert not client.call("ValidateResourceTypeConfig", req).diagnostics
    # plan create
    plan = client.req("PlanResourceChange")
    plan.type_name = "iterative_task"
    plan.prior_state.CopyFrom(dv(None, t))
    plan.proposed_new_state.CopyFrom(dv(config, t))
    plan.config.CopyFrom(dv(config, t))
    pres = client.call("PlanResourceChange", plan)
    planned = cty.decode_msgpack(pres.planned_state.msgpack)
    assert planned["id"] is cty.UNKNOWN and planned["status"] is cty.UNKNOWN
    assert planned["region"] == "us-west" and planned["timeout"] == 86400
    # apply create
    apply = client.req("ApplyResourceChange")
    apply.type_name = "iterative_task"
    apply.prior_state.CopyFrom(dv(None, t))
    apply.planned_state.CopyFrom(pres.planned_state)
    apply.config.CopyFrom(plan.config)
    ares = client.call("ApplyResourceChange", apply)
    assert not [d for d in ares.diagnostics if d.severity == 1], ares.diagnostics
    state = cty.decode_msgpack(ares.new_state.msgpack)
    assert state["id"].startswith("tpi-plugin-test-")
    # read until succeeded
    read = client.req("ReadResource")
    read.type_name = "iterative_task"
    deadline = time.time() + 30
    while True:
        read.current_state.CopyFrom(dv(state, t))
        rres = client.call("ReadResource", read)
        state = cty.decode_msgpack(rres.new_state.msgpack)
        if state["status"] and state["status"].get("succeeded") == 1:
            break
        assert time.time() < deadline, state
        time.sleep(0.1)
    assert "from-plugin" in state["logs"][0]
    # plan a ForceNew change -> requires_replace
    changed = dict(config, machine="m")
    plan.prior_state.CopyFrom(dv(state, t))
    plan.proposed_new_state.CopyFrom(dv(changed, t))
    pres = client.call("PlanResourceChange", plan)
    assert [s.attribute_name for p in pres.requires_replace for s in p.steps] == ["machine"]
    # upgrade state from the JSON Terraform keeps in terraform.tfstate
    up = client.req("UpgradeResourceState")
    up.type_name = "iterative_task"
    up.raw_state.json = json.dumps(state).encode()
    ures = client.call("UpgradeResourceState", up)
    assert cty.decode_msgpack(ures.upgraded_state.msgpack)["id"] == state["id"]
    # import by id
    imp = client.req("ImportResourceState")
    imp.type_name = "iterative_task"
    imp.id = state["id"]
    ires = client.call("ImportResourceState", imp)
    assert cty.decode_msgpack(ires.imported_resources[0].state.msgpack)["cloud"] == "local"
    # destroy
    apply.prior_state.CopyFrom(dv(state, t))
    apply.planned_state.CopyFrom(dv(None, t))
    dres = client.call("ApplyResourceChange", apply)
    assert cty.decode_msgpack(dres.new_state.msgpack) is None
    assert not os.listdir(tmp_path / "state" / "local")


def test_handshake_with_automtls(tmp_path):
    # Terraform side: a client certificate it passes via PLUGIN_CLIENT_CERT
    key, cert = tmp_path / "ck.pem", tmp_path / "cc.pem"
    subprocess.run(["openssl", "req", "-x509", "-newkey", "ec", "-pkeyopt",
                    "ec_paramgen_curve:P-256", "-nodes", "-keyout", str(key), "-out", str(cert),
                    "-days", "1", "-subj", "/CN=localhost", "-addext",
                    "subjectAltName=DNS:localhost"], check=True, capture_output=True)
    env = dict(os.environ, **{MAGIC_COOKIE_KEY: MAGIC_COOKIE_VALUE,
                              "PLUGIN_PROTOCOL_VERSIONS": "5,6",
                              "PLUGIN_CLIENT_CERT": cert.read_text(),
                              "TPI_STATE_ROOT": str(tmp_path / "st")})
    proc = subprocess.Popen([sys.executable, os.path.join(ROOT, "bin", "terraform-provider-iterative")],
                            env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        line = proc.stdout.readline().strip()
        core, app, net, addr, proto, server_cert = line.split("|")
        assert (core, app, net, proto) == ("1", "5", "unix", "grpc")
        der = base64.b64decode(server_cert + "=" * (-len(server_cert) % 4))
        pem = b"-----BEGIN CERTIFICATE-----\n" + base64.encodebytes(der) + \
            b"-----END CERTIFICATE-----\n"
        creds = grpc.ssl_channel_credentials(root_certificates=pem,
                                             private_key=key.read_bytes(),
                                             certificate_chain=cert.read_bytes())
        channel = grpc.secure_channel("unix:" + addr, creds,
                                      options=[("grpc.ssl_target_name_override", "localhost")])
        health = channel.unary_unary("/grpc.health.v1.Health/Check",
                                     request_serializer=lambda b: b,
                                     response_deserializer=lambda b: b)
        assert health(b"\n\x06plugin", timeout=30) == b"\x08\x01"
        res = Client(channel).call("GetSchema", pb.classes("GetSchema")[0]())
        assert "iterative_task" in res.resource_schemas
        shutdown = channel.unary_unary("/plugin.GRPCController/Shutdown",
                                       request_serializer=lambda b: b,
                                       response_deserializer=lambda b: b)
        shutdown(b"", timeout=10)
        assert proc.wait(timeout=30) == 0
    finally:
        if proc.poll() is None:
            proc.kill()


def test_refuses_direct_execution():
    env = {k: v for k, v in os.environ.items() if k != MAGIC_COOKIE_KEY}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bin", "terraform-provider-iterative")],
                       env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "This binary is a plugin" in r.stderr
