"""Machine-script renderer (reference: ``task/common/machine/script.go`` +
``machine-script.sh.tpl``).

The reference renders a cloud-init bash script that installs a systemd unit for the task.
On the node runtime the supervisor is launched directly (``backends/node.py``); this
renderer produces the equivalent *portable* bootstrap for nodes managed outside ``tpi``
(e.g. a scheduler's prolog): it recreates the task directory from base64-embedded pieces --
task script, ``KEY="value"`` environment file, ``export`` credentials file (0600) -- applies
the absolute deadline (``infinity`` or unix seconds, past deadline = nothing runs) and
starts ``tpi-supervisor`` as a systemd user unit when systemd is available, else detached.
"""
from __future__ import annotations

import base64
import json
from typing import Dict, Optional

from ..models.values import Variables
from ..utils.shell import quote

TEMPLATE = """#!/bin/bash
set -e
TPI_TASK_DIRECTORY="${{TPI_TASK_DIRECTORY:-$HOME/.local/state/tpi/node/{task_id}}}"
mkdir -p "$TPI_TASK_DIRECTORY/data" "$TPI_TASK_DIRECTORY/reports" "$TPI_TASK_DIRECTORY/supervisor"
cd "$TPI_TASK_DIRECTORY"

base64 --decode > supervisor/script << END
{task_script}
END
chmod u=rwx,g=rx,o=rx supervisor/script

base64 --decode > supervisor/variables << END
{environment}
END
base64 --decode > supervisor/credentials << END
{credentials}
END
chmod u=rw,g=,o= supervisor/variables supervisor/credentials

TPI_DEADLINE={timeout}
if test "$TPI_DEADLINE" != infinity && (( TPI_DEADLINE <= $(date +%s) )); then
  echo "tpi: deadline passed; not starting" >&2
  exit 0
fi

python3 - "$TPI_TASK_DIRECTORY" "$TPI_DEADLINE" {parallelism} << 'PY'
import json, os, re, shlex, sys
root, deadline, parallelism = sys.argv[1], sys.argv[2], int(sys.argv[3])
env = {{}}
text = open(os.path.join(root, "supervisor", "variables")).read()
for key, value in re.findall(r'(?s)([^\\n=]+)="(.*?)(?<!\\\\)"\\n', text):
    env[key] = value.replace('\\\\"', '"')
for line in open(os.path.join(root, "supervisor", "credentials")):
    line = line.strip()
    if line.startswith("export "):
        key, _, value = shlex.split(line[7:])[0].partition("=")
        env[key] = value
env.setdefault("PATH", os.environ.get("PATH", "/usr/bin:/bin"))
spec = {{"task_id": {task_id_json}, "task_dir": root, "workdir": os.path.join(root, "data"),
        "script": os.path.join(root, "supervisor", "script"), "env": env,
        "deadline": 0 if deadline == "infinity" else float(deadline),
        "parallelism": parallelism, "ranks": [{{"gpus": {gpus_json}}}] * parallelism}}
json.dump(spec, open(os.path.join(root, "supervisor", "spec.json"), "w"))
PY

SUPERVISOR="${{TPI_SUPERVISOR:-{supervisor}}}"
if command -v systemd-run > /dev/null 2>&1 && systemctl --user show-environment > /dev/null 2>&1; then
  systemd-run --user --unit="tpi-task-{task_id}" --collect "$SUPERVISOR" "$TPI_TASK_DIRECTORY/supervisor/spec.json"
else
  "$SUPERVISOR" --daemon "$TPI_TASK_DIRECTORY/supervisor/spec.json" >> supervisor/supervisor.log 2>&1
fi
"""


def render(script: str, credentials: Optional[Dict[str, str]] = None,
           variables: Optional[Variables] = None, timeout: Optional[float] = None,
           task_id: str = "tpi-task", parallelism: int = 1, gpus: str = "",
           supervisor: str = "tpi-supervisor", environ=None) -> str:
    """Render the bootstrap; ``timeout`` is an absolute unix deadline (``None`` = infinity)."""
    environment = ""
    for name, value in sorted((variables or Variables()).enrich(environ or {}).items()):
        environment += '%s="%s"\n' % (name, value.replace('"', '\\"'))
    export = "".join("export %s\n" % quote("%s=%s" % (k, v))
                     for k, v in sorted((credentials or {}).items()))
    b64 = lambda s: base64.b64encode(s.encode()).decode()  # noqa: E731
    return TEMPLATE.format(task_script=b64(script), environment=b64(environment),
                           credentials=b64(export),
                           timeout="infinity" if timeout is None else "%d" % int(timeout),
                           task_id=task_id, task_id_json=json.dumps(task_id),
                           parallelism=int(parallelism), gpus_json=json.dumps(gpus),
                           supervisor=supervisor)
