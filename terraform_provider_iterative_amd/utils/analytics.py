"""Usage telemetry (reference: ``iterative/utils/analytics.go``).

Same payload, user/group identity derivation (scrypt + UUIDv5, bit-compatible), opt-outs
(``ITERATIVE_DO_NOT_TRACK``, ``user_id = do-not-track``, internal CI groups) and endpoint
overrides (``TPI_ANALYTICS_ENDPOINT``/``TPI_ANALYTICS_TOKEN``).  Difference by design: this
framework runs on GPU nodes that usually have no egress, so events are only POSTed when
``TPI_ANALYTICS_ENDPOINT`` is set; otherwise nothing leaves the process.  ``TPI_ANALYTICS_SPOOL``
appends the payloads to a local JSONL file instead (auditable telemetry).
"""
from __future__ import annotations

import json
import logging
import os
import re
import threading
from typing import Any, Dict, List, Optional

from .._version import __version__ as VERSION

log = logging.getLogger("tpi.analytics")

TIMEOUT = 5.0
_pending: List[threading.Thread] = []

EXCLUDED_GROUPS = {
    "dc16cd76-71b7-5afa-bf11-e85e02ee1554",  # deterministic("https://github.com/iterative")
    "b0e229bf-2598-54b7-a3e0-81869cdad579",  # deterministic("https://github.com/iterative-test")
    "d5aaeca4-fe6a-5c72-8aa7-6dcd65974973",  # deterministic("https://gitlab.com/iterative.ai")
    "b6df227b-5b3d-5190-a8fa-d272b617ee6c",  # deterministic("https://gitlab.com/iterative-test")
    "2c6415f0-cb5a-5e52-8c81-c5af4f11715d",  # deterministic("https://bitbucket.com/iterative-ai")
    "c0b86b90-d63c-5fb0-b84d-718d8e15f8d6",  # deterministic("https://bitbucket.com/iterative-test")
}


def deterministic(data: str) -> str:
    import uuid

    ns = uuid.uuid5(uuid.NAMESPACE_DNS, "iterative.ai")
    import hashlib  # scrypt (OpenSSL): only when a CI identity is hashed, not on every start

    dk = hashlib.scrypt(data.encode(), salt=ns.bytes, n=1 << 16, r=8, p=1, dklen=8,
                        maxmem=256 << 20)
    return str(uuid.uuid5(ns, dk.hex()))


def guess_ci(environ=None) -> str:
    environ = os.environ if environ is None else environ
    for var, name in (("GITHUB_SERVER_URL", "github"), ("CI_SERVER_URL", "gitlab"),
                      ("BITBUCKET_WORKSPACE", "bitbucket"), ("TF_BUILD", "azure"),
                      ("CI", "unknown")):
        if var in environ:
            return name
    return ""


def is_ci(environ=None) -> bool:
    return bool(guess_ci(environ))


def group_id(environ=None) -> str:
    environ = os.environ if environ is None else environ
    ci = guess_ci(environ)
    if not ci:
        return ""
    raw = "CI"
    if ci == "github":
        raw = "%s/%s" % (environ.get("GITHUB_SERVER_URL", ""), environ.get("GITHUB_REPOSITORY_OWNER", ""))
    elif ci == "gitlab":
        raw = "%s/%s" % (environ.get("CI_SERVER_URL", ""), environ.get("CI_PROJECT_ROOT_NAMESPACE", ""))
    elif ci == "bitbucket":
        raw = "https://bitbucket.com/%s" % environ.get("BITBUCKET_WORKSPACE", "")
    return deterministic(raw)


def _config_dir(environ) -> str:
    return environ.get("XDG_CONFIG_HOME") or os.path.join(os.path.expanduser("~"), ".config")


def _read_id(path: str) -> str:
    with open(path, "rb") as handle:
        raw = handle.read()
    try:
        data = json.loads(raw)
    except ValueError:
        import uuid

        return str(uuid.UUID(bytes=raw[:16])) if len(raw) >= 16 else raw.decode().strip()
    if isinstance(data, dict) and isinstance(data.get("user_id"), str):
        return data["user_id"]
    raise ValueError("user_id not found or not a string")


def _write_id(path: str, value: str) -> None:
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as handle:
        json.dump({"user_id": value}, handle, indent=2)


def user_id(environ=None) -> str:
    environ = os.environ if environ is None else environ
    ci = guess_ci(environ)
    if ci:
        if ci == "gitlab":
            raw = "%s %s %s" % (environ.get("GITLAB_USER_NAME", ""),
                                environ.get("GITLAB_USER_LOGIN", ""),
                                environ.get("GITLAB_USER_ID", ""))
        elif ci == "bitbucket":
            raw = environ.get("BITBUCKET_STEP_TRIGGERER_UUID", "")
        elif ci == "github":
            raw = "%s %s" % (environ.get("GITHUB_ACTOR", ""), environ.get("GITHUB_ACTOR_ID", ""))
        else:
            import subprocess

            try:
                raw = subprocess.run(["git", "log", "-1", "--pretty=format:'%ae'"],
                                     capture_output=True, text=True, timeout=5).stdout
            except OSError:
                raw = "CI"
        return deterministic(raw)
    base = _config_dir(environ)
    old = os.path.join(base, "dvc", "user_id")
    new = os.path.join(base, "iterative", "telemetry")
    import uuid

    ident = str(uuid.uuid4())
    if not os.path.exists(new):
        if os.path.exists(old):
            ident = _read_id(old)
        _write_id(new, ident)
    else:
        ident = _read_id(new)
    if not os.path.exists(old) and ident != "do-not-track":
        _write_id(old, ident)
    return ident


_TS = re.compile(r"\d{4}-\d{2}-\d{2}[ T]\d{2}:\d{2}:\d{2}")


def task_duration(logs: str) -> float:
    import datetime as dt

    matches = _TS.findall(logs)
    if len(matches) < 2:
        return 0.0
    parse = lambda s: dt.datetime.strptime(s.replace("T", " "), "%Y-%m-%d %H:%M:%S")  # noqa
    return (parse(matches[-1]) - parse(matches[0])).total_seconds()


def resource_data(data: Optional[Dict[str, Any]]) -> Dict[str, Any]:
    if not data:
        return {}
    logs = data.get("logs") or []
    spot = float(data.get("spot", -1) or 0) if data.get("spot") is not None else -1.0
    return {"cloud": data.get("cloud", ""), "cloud_region": data.get("region", ""),
            "cloud_machine": data.get("machine", ""), "cloud_disk_size": data.get("disk_size", -1),
            "cloud_spot": spot, "cloud_spot_auto": spot == 0.0,
            "task_status": data.get("status") or {}, "task_duration": task_duration("".join(logs)),
            "task_resumed": len(logs) > 1}


def payload(action: str, error: Optional[BaseException], extra: Dict[str, Any],
            environ=None) -> Dict[str, Any]:
    import platform

    environ = os.environ if environ is None else environ
    extra = dict(extra)
    extra["ci"] = guess_ci(environ)
    extra["terraform_version"] = environ.get("TPI_TERRAFORM_VERSION", "")
    body = {"user_id": user_id(environ), "group_id": group_id(environ), "action": action,
            "interface": "cli", "tool_name": "tpi", "tool_source": "terraform",
            "tool_version": VERSION, "os_name": platform.system().lower(),
            "os_version": platform.release(), "backend": extra.get("cloud"), "extra": extra}
    if error is not None:
        body["error"] = type(error).__name__  # type only: messages may be sensitive
    return body


def _post(body: Dict[str, Any], endpoint: str, token: str) -> None:
    import urllib.request

    req = urllib.request.Request(endpoint, data=json.dumps(body).encode(), method="POST",
                                 headers={"Content-Type": "application/json",
                                          "X-Auth-Token": token})
    try:
        urllib.request.urlopen(req, timeout=TIMEOUT).close()
    except Exception as exc:  # telemetry must never break the tool
        log.debug("analytics: %s", exc)


def send_event(action: str, error: Optional[BaseException], data: Optional[Dict[str, Any]],
               environ=None) -> Optional[Dict[str, Any]]:
    environ = os.environ if environ is None else environ
    if "ITERATIVE_DO_NOT_TRACK" in environ:
        return None
    if environ.get("GITHUB_REPOSITORY", "").startswith("iterative/"):
        return None
    endpoint = environ.get("TPI_ANALYTICS_ENDPOINT")
    spool = environ.get("TPI_ANALYTICS_SPOOL")
    if not endpoint and not spool:
        return None
    try:
        body = payload(action, error, resource_data(data), environ)
    except Exception as exc:
        log.debug("analytics: payload failed: %s", exc)
        return None
    if body["group_id"] in EXCLUDED_GROUPS or body["user_id"] == "do-not-track":
        return None
    if spool:
        with open(spool, "a") as handle:
            handle.write(json.dumps(body) + "\n")
    if endpoint:
        t = threading.Thread(target=_post, args=(body, endpoint,
                                                 environ.get("TPI_ANALYTICS_TOKEN", "")),
                             daemon=True)
        t.start()
        _pending.append(t)
    return body


def wait_for_analytics(timeout: float = TIMEOUT) -> None:
    while _pending:
        _pending.pop().join(timeout)
