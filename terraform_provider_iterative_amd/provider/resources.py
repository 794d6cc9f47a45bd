"""Resource implementations: ``iterative_task``, ``iterative_machine``, ``iterative_cml_runner``.

Each function takes the resource's (normalized) attribute dict and returns the new state
attributes plus diagnostics, the way the reference's ``schema.Resource`` Create/Read/Delete
contexts update ``*schema.ResourceData``:

* ``iterative/resource_task.go:206-446``    task create/read/delete/build
* ``iterative/resource_machine.go:148-295`` machine create/delete (read is a no-op)
* ``iterative/resource_runner.go:196-485``  runner create (wait for ``{"status":"ready"}``)
"""
from __future__ import annotations

import base64
import datetime as _dt
import logging
import os
import time
from typing import Any, Dict, List, Optional, Tuple

from ..utils.record import field, record
from .. import backends
from ..models.cloud import Cloud, Timeouts, PROVIDER_LOCAL, PROVIDER_MI355X
from ..models.schema import get_schema
from ..models.values import (Environment, Firewall, FirewallRule, NotImplementedErr,
                             RemoteStorage, Size, Task as TaskSpec, Variables)
from ..utils import analytics
from ..utils.identifier import (new_deterministic_identifier, new_random_identifier,
                                parse_identifier)
from ..utils.shell import quote as shell_quote

log = logging.getLogger("tpi")

CI_FORWARD = ("CI", "CI_*", "GITHUB_*", "BITBUCKET_*", "CML_*", "REPO_TOKEN")
LOG_TPL = ("%s may take several minutes (consider increasing `timeout` "
           "https://registry.terraform.io/providers/iterative/iterative/latest/docs/resources/"
           "task#timeout). Please wait.")


@record
class Diagnostic:
    severity: str  # "error" | "warning"
    summary: str
    detail: str = ""


@record
class Result:
    id: str
    state: Dict[str, Any]
    diagnostics: List[Diagnostic] = field(default_factory=list)

    @property
    def ok(self) -> bool:
        return not any(d.severity == "error" for d in self.diagnostics)


def _timeouts(resource_type: str, overrides: Optional[Dict[str, float]] = None) -> Timeouts:
    base = dict(get_schema(resource_type).timeouts)
    base.update({k: v for k, v in (overrides or {}).items() if v})
    return Timeouts(create=base.get("create", 900), read=base.get("read", 180),
                    update=base.get("update", 180), delete=base.get("delete", 900))


# ---- iterative_task ---------------------------------------------------------------------------

def _split_container(cloud: str, container: str) -> Tuple[str, str]:
    """rclone ``bucket.Split`` for remote clouds; node providers take a directory path."""
    if cloud in (PROVIDER_LOCAL, PROVIDER_MI355X) or container.startswith(":"):
        return container, ""
    container = container.lstrip("/")
    bucket, _, path = container.partition("/")
    return bucket, path


def build_task(data: Dict[str, Any], resource_id: str = "",
               timeouts: Optional[Dict[str, float]] = None, environ=None) -> backends.Task:
    """``resourceTaskBuild`` (``resource_task.go:328-446``)."""
    environ = os.environ if environ is None else environ
    variables = Variables()
    for name, value in (data.get("environment") or {}).items():
        variables[name] = value if value != "" else None
    variables["TPI_TASK"] = "true"
    for pattern in CI_FORWARD:
        variables[pattern] = None
    cloud = Cloud(provider=data["cloud"], region=data.get("region") or "us-west",
                  timeouts=_timeouts("iterative_task", timeouts),
                  tags=dict(data.get("tags") or {}))
    directory = directory_out = ""
    excludes: List[str] = []
    remote = None
    storage = (data.get("storage") or [])
    if storage:
        block = storage[0]
        directory = block.get("workdir") or ""
        directory_out = block.get("output") or ""
        if os.path.isabs(directory_out) or directory_out.startswith("../"):
            raise ValueError("storage.output must be inside storage.workdir")
        excludes = list(block.get("exclude") or [])
        if block.get("container"):
            container, path = _split_container(cloud.provider, block["container"])
            remote = RemoteStorage(container, path, {str(k): str(v) for k, v in
                                                     (block.get("container_opts") or {}).items()})
    task = TaskSpec(
        size=Size(machine=data.get("machine") or "m", storage=int(data.get("disk_size", -1))),
        environment=Environment(image=data.get("image") or "ubuntu",
                                script=data.get("script") or "", variables=variables,
                                directory=directory, directory_out=directory_out,
                                exclude_list=excludes,
                                timeout=float(data.get("timeout") or 0)),
        firewall=Firewall(ingress=FirewallRule(ports=[22, 80])),
        remote_storage=remote, spot=float(data.get("spot", -1)),
        parallelism=int(data.get("parallelism") or 1),
        permission_set=data.get("permission_set") or "")
    try:
        ident = parse_identifier(resource_id)
    except ValueError:
        name = data.get("name") or ""
        if name:
            try:
                ident = parse_identifier(name)
            except ValueError:
                ident = new_deterministic_identifier(name)
        elif environ.get("GITHUB_RUN_ID"):
            ident = new_deterministic_identifier(environ["GITHUB_RUN_ID"])
        elif environ.get("CI_PIPELINE_ID"):
            ident = new_deterministic_identifier(environ["CI_PIPELINE_ID"])
        elif environ.get("BITBUCKET_STEP_TRIGGERER_UUID"):
            ident = new_deterministic_identifier(environ["BITBUCKET_STEP_TRIGGERER_UUID"])
        else:
            ident = new_random_identifier("")
    return backends.new(cloud, ident, task)


def task_create(data: Dict[str, Any], timeouts: Optional[Dict[str, float]] = None) -> Result:
    log.info(LOG_TPL, "Creation")
    diags: List[Diagnostic] = []
    if float(data.get("spot", -1)) > 0:
        log.warning("Setting a maximum price `spot=%f` USD/h. Consider using auto-pricing "
                    "(`spot=0`) instead.", float(data["spot"]))
    try:
        task = build_task(data, "", timeouts)
    except Exception as error:
        analytics.send_event("task/apply", error, data)
        return Result("", dict(data), [Diagnostic("error", str(error))])
    rid = task.get_identifier().long()
    err = None
    try:
        task.create()
    except Exception as error:  # roll back like resource_task.go:221-229
        err = error
        diags.append(Diagnostic("error", str(error)))
        try:
            task.delete()
            diags.append(Diagnostic("error", "failed to create"))
            rid = ""
        except Exception as cleanup:
            diags.append(Diagnostic("error", str(cleanup)))
    analytics.send_event("task/apply", err, data)
    state = dict(data)
    state["id"] = rid
    if rid:
        read = task_read(state, timeouts, send=False)
        state = read.state
        diags.extend(d for d in read.diagnostics if d.severity == "error")
    return Result(rid, state, diags)


def task_read(data: Dict[str, Any], timeouts: Optional[Dict[str, float]] = None,
              send: bool = True) -> Result:
    rid = data.get("id") or ""
    state = dict(data)
    try:
        task = build_task(data, rid, timeouts)
        task.read()
    except Exception as error:
        if send:
            analytics.send_event("task/read", error, data)
        return Result(rid, state, [Diagnostic("warning", str(error))])
    try:
        key = task.get_key_pair()
        state["ssh_public_key"], state["ssh_private_key"] = key.public_string(), key.private_string()
    except NotImplementedErr:
        pass
    state["addresses"] = list(task.get_addresses())
    state["events"] = [e.format_resource() for e in task.events()]
    state["status"] = dict(task.status())
    state["logs"] = list(task.logs())
    state["id"] = task.get_identifier().long()
    if send:
        analytics.send_event("task/read", None, state)
    return Result(state["id"], state)


def task_delete(data: Dict[str, Any], timeouts: Optional[Dict[str, float]] = None) -> Result:
    log.info(LOG_TPL, "Destruction")
    rid = data.get("id") or ""
    err = None
    diags = []
    try:
        task = build_task(data, rid, timeouts)
        task.delete()
    except Exception as error:
        err = error
        diags.append(Diagnostic("error", str(error)))
    analytics.send_event("task/destroy", err, data)
    return Result(rid if err else "", dict(data), diags)


# ---- iterative_machine / iterative_cml_runner ---------------------------------------------------

def _set_id(data: Dict[str, Any]) -> str:
    """``utils.SetId``: random identifier with the ``cml-`` prefix."""
    if data.get("id"):
        return data["id"]
    ident = new_random_identifier(data.get("name") or "")
    return ident.long().replace("tpi-", "cml-", 1)


def _machine_task(data: Dict[str, Any], rid: str, script: str) -> backends.Task:
    cloud_name = data.get("cloud") or ""
    if cloud_name in ("azure",):
        cloud_name = "az"
    if cloud_name in ("kubernetes",):
        cloud_name = "k8s"
    machine = data.get("instance_type") or "m"
    gpu = (data.get("instance_gpu") or "").strip()
    if gpu:
        machine = machine + "+" + ("mi355x" if gpu in ("mi355x", "tesla", "v100", "k80", "t4",
                                                       "gpu") else gpu)
    cloud = Cloud(provider=cloud_name, region=data.get("region") or "us-west",
                  tags=dict(data.get("metadata") or {}))
    spec = TaskSpec(size=Size(machine=machine, storage=int(data.get("instance_hdd_size") or 35)),
                    environment=Environment(image=data.get("image") or "ubuntu", script=script,
                                            variables=Variables({"TPI_MACHINE": "true"})),
                    spot=0.0 if data.get("spot") else -1.0,
                    permission_set=data.get("instance_permission_set") or "")
    return backends.new(cloud, parse_identifier(rid), spec)


def machine_create(data: Dict[str, Any], timeouts: Optional[Dict[str, float]] = None) -> Result:
    state = dict(data)
    rid = _set_id(state)
    state["id"] = rid
    diags: List[Diagnostic] = []
    try:
        if not state.get("ssh_private"):
            from ..utils.ssh import private_pem  # machines only: keep task CLIs light

            state["ssh_private"] = private_pem()
        from ..utils.ssh import public_from_private_pem

        state["ssh_public"] = public_from_private_pem(state["ssh_private"])
    except Exception as error:
        return Result("", state, [Diagnostic("error", "Failed creating the key pair: %s" % error)])
    script = state.get("startup_script") or "#!/bin/bash"
    state["startup_script"] = base64.b64encode(script.encode()).decode()
    cloud = state.get("cloud") or ""
    if state.get("instance_permission_set") and cloud in ("kubernetes", "k8s"):
        return Result("", state, [Diagnostic(
            "error", "instance_permission_set is not yet supported in " + cloud)])
    if not cloud:
        return Result("", state, [Diagnostic("error", "Unknown cloud: %s" % cloud)])
    try:
        task = _machine_task(state, rid, script)
        task.create()
    except Exception as error:
        diags.append(Diagnostic("error", "Failed creating the machine: %s" % error))
        machine_delete(state)
        return Result("", state, diags)
    from ..backends.node import node_address

    state["instance_ip"] = node_address()
    state["instance_launch_time"] = _dt.datetime.now(_dt.timezone.utc).strftime(
        "%Y-%m-%dT%H:%M:%SZ")
    return Result(rid, state, diags)


def machine_read(data: Dict[str, Any], timeouts=None) -> Result:
    return Result(data.get("id") or "", dict(data))  # resource_machine.go:280-282


def machine_delete(data: Dict[str, Any], timeouts=None) -> Result:
    rid = data.get("id") or ""
    if not data.get("cloud"):
        return Result(rid, dict(data), [Diagnostic("error", "Unknown cloud: ")])
    try:
        _machine_task(data, rid, "").delete()
    except Exception as error:
        return Result(rid, dict(data), [Diagnostic("error", "Failed disposing the machine: %s"
                                                   % error)])
    return Result("", dict(data))


def machine_logs(data: Dict[str, Any]) -> str:
    task = _machine_task(data, data["id"], "")
    return "\n".join(task.logs())


RUNNER_TEMPLATE = """#!/bin/sh
# CML runner on the node-local runtime ({cloud}); generated by terraform-provider-iterative_amd
{exports}{startup}
HOME="$(mktemp -d)" exec $(command -v cml-runner || echo "$(command -v cml-internal || echo cml) runner") \\
{flags}
"""

# Credentials the runner's own `cml`/`leo` calls need, per cloud (resource_runner.go:329-349).
RUNNER_CREDENTIALS = {
    "aws": ("AWS_SECRET_ACCESS_KEY", "AWS_ACCESS_KEY_ID", "AWS_SESSION_TOKEN"),
    "azure": ("AZURE_CLIENT_ID", "AZURE_CLIENT_SECRET", "AZURE_SUBSCRIPTION_ID",
              "AZURE_TENANT_ID"),
    "gcp": ("GOOGLE_APPLICATION_CREDENTIALS_DATA", "CML_GCP_ACCESS_TOKEN"),
    "kubernetes": ("KUBERNETES_CONFIGURATION",),
    "local": ("TPI_STATE_ROOT",),
    "mi355x": ("TPI_STATE_ROOT", "TPI_MI355X_GPUS"),
}


def runner_credentials(cloud: str, environ=None) -> List[Tuple[str, str]]:
    """(name, value) exports for the runner script.  GCP credentials are only forwarded when
    they parse as a credentials JSON document, like ``gcp.LoadGCPCredentials``."""
    import json

    environ = os.environ if environ is None else environ
    out = []
    for name in RUNNER_CREDENTIALS.get(cloud or "", ()):
        value = environ.get(name, "")
        if name == "GOOGLE_APPLICATION_CREDENTIALS_DATA" and value:
            try:
                json.loads(value)
            except ValueError:
                value = ""
        if cloud in ("local", "mi355x") and not value:
            continue  # node defaults apply
        out.append((name, value))
    return out


def render_runner_script(data: Dict[str, Any], environ=None) -> str:
    """Runner startup script (the node equivalent of ``renderScript``,
    ``resource_runner.go:298-400``): decoded user startup script + ``cml runner`` flags."""
    startup = ""
    if data.get("startup_script"):
        startup = base64.b64decode(data["startup_script"]).decode()
    flags = []
    for key, flag in (("name", "--name"), ("labels", "--labels"),
                      ("idle_timeout", "--idle-timeout"), ("driver", "--driver"),
                      ("repo", "--repo"), ("token", "--token")):
        if data.get(key) not in (None, ""):
            flags.append("%s %s" % (flag, shell_quote(str(data[key]))))
    if data.get("single"):
        flags.append("--single")
    for volume in data.get("docker_volumes") or []:
        flags.append("--docker-volumes %s" % shell_quote(volume))
    if data.get("tf_resource"):
        flags.append("--tf-resource %s" % shell_quote(data["tf_resource"]))
    exports = "".join("export %s=%s\n" % (name, shell_quote(value))
                      for name, value in runner_credentials(data.get("cloud") or "", environ))
    return RUNNER_TEMPLATE.format(cloud=data.get("cloud") or "-", startup=startup,
                                  exports=exports,
                                  flags=" \\\n".join("  " + f for f in flags))


def _go_json(value) -> str:
    """``encoding/json.Marshal`` byte-for-byte: compact, UTF-8, HTML-safe escapes."""
    import json

    text = json.dumps(value, separators=(",", ":"), ensure_ascii=False)
    for char, esc in (("<", "\\u003c"), (">", "\\u003e"), ("&", "\\u0026"),
                      ("\u2028", "\\u2028"), ("\u2029", "\\u2029")):
        text = text.replace(char, esc)
    return text


def runner_tf_resource(data: Dict[str, Any], rid: str) -> str:
    """Synthetic state resource handed to ``cml runner --tf-resource`` (``ResourceType``,
    ``resource_runner.go:405-531``) so the runner can destroy itself via the state.  Field
    order and encoding follow the Go structs, so the base64 matches the reference's."""
    attrs = {"name": rid, "labels": "", "idle_timeout": int(data.get("idle_timeout") or 0),
             "repo": "", "token": "", "driver": "", "cloud": data.get("cloud") or "",
             "spot": bool(data.get("spot")), "custom_data": "", "id": rid, "image": "",
             "instance_gpu": "", "instance_hdd_size": int(data.get("instance_hdd_size") or 0),
             "instance_ip": "", "instance_launch_time": "", "instance_type": "",
             "region": data.get("region") or "", "ssh_name": "", "ssh_private": "",
             "ssh_public": "", "aws_security_group": ""}
    resource = {"mode": "managed", "type": "iterative_cml_runner", "name": "runner",
                "provider": 'provider["registry.terraform.io/iterative/iterative"]',
                "instances": [{"private": "", "schema_version": 0, "attributes": attrs}]}
    return base64.b64encode(_go_json(resource).encode()).decode()


def runner_create(data: Dict[str, Any], timeouts: Optional[Dict[str, float]] = None,
                  environ=None, poll: float = 1.0) -> Result:
    environ = os.environ if environ is None else environ
    state = dict(data)
    rid = _set_id(state)
    state["id"] = rid
    if not state.get("token") and environ.get("CML_TOKEN"):
        state["token"] = environ["CML_TOKEN"]
    if not state.get("token"):
        return Result("", state, [Diagnostic("error", "Token not found nor in tf file nor in "
                                             "env CML_TOKEN")])
    diags: List[Diagnostic] = []
    if state.get("instance_gpu") == "tesla":
        diags.append(Diagnostic("warning", "GPU model 'tesla' has been deprecated; please use "
                                "'v100' instead"))
        state["instance_gpu"] = "v100"
    if not state.get("cloud"):
        return Result("", state, [Diagnostic("error", "Local runner not yet implemented")])
    render = dict(state)
    render["name"] = rid
    render["tf_resource"] = runner_tf_resource(state, rid)
    render["startup_script"] = base64.b64encode(
        (state.get("startup_script") or "").encode()).decode()
    state["startup_script"] = render_runner_script(render)
    created = machine_create(state, timeouts)
    diags.extend(created.diagnostics)
    if not created.ok:
        return Result("", created.state, diags)
    state = created.state
    from ..utils.runner_status import has_status

    budget = _timeouts("iterative_cml_runner", timeouts).create - 60.0
    deadline = time.time() + max(budget, 1.0)
    logs = ""
    while time.time() < deadline:
        logs = machine_logs(state)
        if has_status(logs, "terminated"):
            break
        if has_status(logs, "ready"):
            return Result(rid, state, diags)
        time.sleep(poll)
    machine_delete(state)
    diags.append(Diagnostic("error", "Error checking the runner status", logs))
    return Result("", state, diags)


def runner_delete(data: Dict[str, Any], timeouts=None) -> Result:
    return machine_delete(data, timeouts)


HANDLERS = {
    "iterative_task": {"create": task_create, "read": task_read, "delete": task_delete},
    "iterative_machine": {"create": machine_create, "read": machine_read,
                          "delete": machine_delete},
    "iterative_cml_runner": {"create": runner_create, "read": machine_read,
                             "delete": runner_delete},
}


def handler(resource_type: str, op: str):
    from ..models.schema import ALIASES

    return HANDLERS[ALIASES.get(resource_type, resource_type)][op]
