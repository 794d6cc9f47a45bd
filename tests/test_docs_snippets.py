"""The Python snippet of ``docs/guides/migrating.md`` runs as written (on CPU here): a local
task whose rank SIGTERMs itself mid-loop resumes from the checkpoint and finishes."""
import os
import re
import sys

from terraform_provider_iterative_amd import backends
from terraform_provider_iterative_amd.models.cloud import Cloud, Credentials, NodeCredentials
from terraform_provider_iterative_amd.models.values import Environment, Task, Variables
from terraform_provider_iterative_amd.utils.identifier import new_deterministic_identifier

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PRELUDE = r'''#!%(python)s
import os, signal, sys
sys.path.insert(0, %(root)r)
import torch
torch.set_num_threads(1)
torch.manual_seed(0)
model = torch.nn.Linear(8, 8)
opt = torch.optim.AdamW(model.parameters(), lr=1e-2)
model(torch.zeros(1, 8)).sum().backward()
opt.step()                                    # optimizer state exists from here on
total_steps = 6
first = os.environ.get("TPI_RESTART_COUNT", "0") == "0"

def train_one_step(model, opt):
    opt.zero_grad()
    model(torch.randn(4, 8)).pow(2).mean().backward()
    opt.step()
    if first and int(step.item()) == 2:       # preempted inside step 3 of the first run
        os.kill(os.getpid(), signal.SIGTERM)
'''


def _snippet() -> str:
    text = open(os.path.join(ROOT, "docs", "guides", "migrating.md")).read()
    blocks = re.findall(r"```python\n(.*?)```", text, re.S)
    assert len(blocks) == 1, "the guide has one Python snippet"
    return blocks[0].replace('device="cuda"', 'device="cpu"')


def test_migration_guide_snippet_resumes_after_a_preemption(tmp_path):
    code = (PRELUDE % {"python": sys.executable, "root": ROOT}) + _snippet() + \
        '\nprint("resumed at", meta_start, "final", int(step.item()), flush=True)\n'
    # the snippet's resume() result, recorded where it is taken
    code = code.replace("state.resume()", "meta_start = (state.resume() or {}).get('step')", 1)
    cloud = Cloud(provider="local",
                  credentials=Credentials(node=NodeCredentials(state_root=str(tmp_path / "st"))))
    spec = Task(environment=Environment(script=code, timeout=300,
                                        variables=Variables({"TPI_TASK": "true"})))
    task = backends.new(cloud, new_deterministic_identifier("docs-snippet"), spec)
    task.create()
    status = task.wait(240)
    logs = task.logs()
    task.delete()
    assert status["succeeded"] == 1, (status, logs)
    assert len(logs) == 2, logs  # preempted once, resumed once
    assert "resumed at None final 6" not in logs[0]
    line = [l for l in logs[1].splitlines() if "resumed at" in l]
    assert line, logs
    resumed = int(line[0].split("resumed at ")[1].split()[0])
    assert resumed == 3, logs  # saved at the boundary that ends step 3
    assert line[0].endswith("final 6"), logs
