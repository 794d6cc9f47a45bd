"""iterative_machine / iterative_cml_runner on the node runtime and task build rules
(resource_task.go:328-446, resource_machine.go, resource_runner.go, resource_runner_test.go)."""
import base64
import json
import os
import stat

import pytest

from terraform_provider_iterative_amd.models.schema import SchemaError, normalize
from terraform_provider_iterative_amd.provider import resources


@pytest.fixture(autouse=True)
def state_root(tmp_path, monkeypatch):
    monkeypatch.setenv("TPI_STATE_ROOT", str(tmp_path / "state"))
    for var in ("GITHUB_RUN_ID", "CI_PIPELINE_ID", "BITBUCKET_STEP_TRIGGERER_UUID"):
        monkeypatch.delenv(var, raising=False)
    return tmp_path / "state"


def test_schema_defaults_and_validation():
    d = normalize("iterative_task", {"cloud": "local", "script": "#!/bin/sh\n"})
    assert d["region"] == "us-west" and d["machine"] == "m" and d["spot"] == -1.0
    assert d["timeout"] == 86400 and d["parallelism"] == 1 and d["image"] == "ubuntu"
    assert d["storage"] == [] and d["status"] is None
    with pytest.raises(SchemaError):
        normalize("iterative_task", {"cloud": "local"})
    with pytest.raises(SchemaError):
        normalize("iterative_task", {"cloud": "local", "script": "x", "bogus": 1})
    with pytest.raises(SchemaError):
        normalize("iterative_task", {"cloud": "local", "script": "x", "parallelism": "two"})
    s = normalize("iterative_task", {"cloud": "local", "script": "x",
                                     "storage": [{"workdir": "."}]})
    assert s["storage"] == [{"workdir": ".", "output": "", "container": "",
                             "container_opts": None, "exclude": None}]
    assert normalize("iterative_runner", {"repo": "r", "driver": "github"})["labels"] == "cml"


def test_task_id_precedence(monkeypatch):
    base = normalize("iterative_task", {"cloud": "local", "script": "#!/bin/sh\n"})
    t = resources.build_task(dict(base, name="my task"))
    assert t.get_identifier().long().startswith("tpi-my-task-")
    parsed = resources.build_task(dict(base, name="tpi-test-3z4xlzwq-3u0vweb4"))
    assert parsed.get_identifier().long() == "tpi-test-3z4xlzwq-3u0vweb4"
    monkeypatch.setenv("GITHUB_RUN_ID", "12345")
    gh = resources.build_task(base)
    assert gh.get_identifier().long().startswith("tpi-12345-")
    existing = resources.build_task(base, resource_id="tpi-test-3z4xlzwq-3u0vweb4")
    assert existing.get_identifier().long() == "tpi-test-3z4xlzwq-3u0vweb4"


def test_task_build_rules():
    base = normalize("iterative_task", {"cloud": "local", "script": "#!/bin/sh\n",
                                        "environment": {"A": "1", "INHERIT": ""},
                                        "storage": [{"output": "../escape"}]})
    with pytest.raises(ValueError, match="inside storage.workdir"):
        resources.build_task(base)
    ok = dict(base, storage=[{"workdir": ".", "output": "out", "container": "/data/bucket",
                              "container_opts": {"k": "v"}, "exclude": ["x"]}])
    t = resources.build_task(ok)
    env = t.spec.environment.variables
    assert env["A"] == "1" and env["INHERIT"] is None and env["TPI_TASK"] == "true"
    assert env["GITHUB_*"] is None and "REPO_TOKEN" in env
    assert t.spec.firewall.ingress.ports == [22, 80]
    assert t.remote.container == "/data/bucket" and t.data_dir == "/data/bucket"
    remote = resources.build_task(dict(ok, cloud="aws"))
    assert remote.task.remote_storage.container == "data"
    assert remote.task.remote_storage.path == "bucket"


def test_remote_cloud_diagnostic():
    data = normalize("iterative_task", {"cloud": "aws", "script": "#!/bin/sh\n"})
    result = resources.task_create(data)
    assert not result.ok and "remote provider" in result.diagnostics[0].summary


def test_machine_create_delete(state_root):
    data = normalize("iterative_machine", {"cloud": "local", "name": "box",
                                           "startup_script": "#!/bin/sh\necho machine-up\n",
                                           "instance_type": "s"})
    result = resources.machine_create(data)
    assert result.ok, result.diagnostics
    st = result.state
    assert st["id"].startswith("cml-box-")
    assert st["ssh_public"].startswith("ssh-rsa ")
    assert st["ssh_private"].startswith("-----BEGIN RSA PRIVATE KEY-----")
    assert base64.b64decode(st["startup_script"]).decode().endswith("echo machine-up\n")
    assert st["instance_ip"] and st["instance_launch_time"].endswith("Z")
    import time

    deadline = time.time() + 10
    while "machine-up" not in resources.machine_logs(st) and time.time() < deadline:
        time.sleep(0.05)
    assert "machine-up" in resources.machine_logs(st)
    assert resources.machine_delete(st).ok
    assert not os.listdir(os.path.join(str(state_root), "local"))


def test_runner_script_rendering():
    script = resources.render_runner_script({
        "startup_script": base64.b64encode(b'echo "hello world"\necho "bye world"').decode(),
        "docker_volumes": ["/one/one.txt:/one/one.txt", "/two:/two"], "single": True,
        "name": 'value with "quotes" and spaces', "labels": "cml,gpu", "idle_timeout": 11,
        "driver": "github", "repo": "https://github.com/o/r", "token": "t0k"})
    assert 'echo "hello world"\necho "bye world"' in script
    assert "--docker-volumes /one/one.txt:/one/one.txt" in script
    assert "--docker-volumes /two:/two" in script
    assert "--name 'value with \"quotes\" and spaces'" in script
    assert "--single" in script and "--idle-timeout 11" in script
    tf = json.loads(base64.b64decode(resources.runner_tf_resource({"cloud": "mi355x"}, "cml-x")))
    assert tf["type"] == "iterative_cml_runner" and tf["instances"][0]["attributes"]["id"] == "cml-x"


def test_runner_waits_for_ready(tmp_path, monkeypatch):
    bindir = tmp_path / "bin"
    bindir.mkdir()
    cml = bindir / "cml-runner"
    cml.write_text('#!/bin/sh\necho "args: $*"\necho \'{"level":"info","status":"ready"}\'\n'
                   "sleep 30\n")
    cml.chmod(cml.stat().st_mode | stat.S_IEXEC)
    monkeypatch.setenv("PATH", "%s:%s" % (bindir, os.environ["PATH"]))
    monkeypatch.setenv("CML_TOKEN", "tok")
    data = normalize("iterative_cml_runner", {"repo": "https://github.com/o/r",
                                              "driver": "github", "cloud": "local",
                                              "instance_type": "s"})
    result = resources.runner_create(data, poll=0.05)
    assert result.ok, [d.summary for d in result.diagnostics]
    logs = resources.machine_logs(result.state)
    assert "--repo https://github.com/o/r" in logs and "--token tok" in logs
    assert resources.runner_delete(result.state).ok


def test_runner_requires_token(monkeypatch):
    monkeypatch.delenv("CML_TOKEN", raising=False)
    data = normalize("iterative_cml_runner", {"repo": "r", "driver": "github", "cloud": "local"})
    result = resources.runner_create(data)
    assert not result.ok and "Token not found" in result.diagnostics[0].summary


# Environment / schema fixtures of the reference's runner golden test
# (iterative/resource_runner_test.go:56-89); the goldens are copied from its testdata.
_GOLDEN_ENV = {
    "AWS_SECRET_ACCESS_KEY": '0 value with "quotes" and spaces',
    "AWS_ACCESS_KEY_ID": '1 value with "quotes" and spaces',
    "AWS_SESSION_TOKEN": '2 value with "quotes" and spaces',
    "AZURE_CLIENT_ID": '3 value with "quotes" and spaces',
    "AZURE_CLIENT_SECRET": '4 value with "quotes" and spaces',
    "AZURE_SUBSCRIPTION_ID": '5 value with "quotes" and spaces',
    "AZURE_TENANT_ID": '6 value with "quotes" and spaces',
    "GOOGLE_APPLICATION_CREDENTIALS_DATA": '7 value with "quotes" and spaces',
    "KUBERNETES_CONFIGURATION": '8 value with "quotes" and spaces',
}
_GOLDEN_DIR = os.path.join(os.path.dirname(__file__), "testdata", "runner")


def _golden(cloud):
    with open(os.path.join(_GOLDEN_DIR, "script_template_cloud_%s.golden" % cloud)) as handle:
        return handle.read()


@pytest.mark.parametrize("cloud", ["aws", "azure", "gcp", "kubernetes", "invalid"])
def test_runner_golden_parity(cloud):
    """Credential exports and the --tf-resource payload match the reference's goldens."""
    golden = _golden(cloud)
    data = {"cloud": cloud, "region": '9 value with "quotes" and spaces',
            "name": "", "single": True, "idle_timeout": 11, "instance_hdd_size": 12,
            "token": '13 value with "quotes" and spaces',
            "repo": '14 value with "quotes" and spaces',
            "driver": '15 value with "quotes" and spaces',
            "labels": '16 value with "quotes" and spaces'}
    tf = resources.runner_tf_resource(data, "")
    assert "--tf-resource " + tf in golden  # byte-identical JSON + base64
    script = resources.render_runner_script(dict(data, tf_resource=tf), _GOLDEN_ENV)
    exports = [line for line in script.splitlines() if line.startswith("export ")]
    want = [line for line in golden.splitlines()
            if line.startswith("export ") and "DEBIAN_FRONTEND" not in line]
    assert exports == want
    for flag in ("--labels", "--idle-timeout", "--driver", "--repo", "--token"):
        mine = [line.strip(" \\") for line in script.splitlines() if line.strip().startswith(flag)]
        theirs = [line.strip(" \\") for line in golden.splitlines()
                  if line.strip().startswith(flag)]
        assert mine == theirs, flag


def test_permission_set_grammar():
    from terraform_provider_iterative_amd.models.permissions import (PermissionSetError,
                                                                     parse_permission_set)

    # task/az/resources/data_source_permission_set_test.go vectors
    ok = ("/subscriptions/cse78759-ef49-49f7-b371-f6841fa82182/resourceGroups/resource-group"
          "/providers/Microsoft.ManagedIdentity/userAssignedIdentities/managed-identity")
    assert parse_permission_set("az", ok + ", ")["user_assigned_identities"] == [ok]
    with pytest.raises(PermissionSetError) as err:
        parse_permission_set("az", "/subscriptions/no-valid")
    assert str(err.value) == 'invalid user-assigned identity id: "/subscriptions/no-valid"'
    assert parse_permission_set("aws", "arn:aws:iam::123:instance-profile/x")["arn"]
    with pytest.raises(PermissionSetError, match="invalid IAM Instance Profile"):
        parse_permission_set("aws", "role/x")
    gcp = parse_permission_set("gcp", "sa@p.iam.gserviceaccount.com,scopes=storage-rw,custom")
    assert gcp["scopes"] == ["https://www.googleapis.com/auth/devstorage.read_write", "custom"]
    with pytest.raises(PermissionSetError, match="at least one scope"):
        parse_permission_set("gcp", "sa@p")
    assert parse_permission_set("k8s", "runner-sa") == {"service_account": "runner-sa"}
    assert parse_permission_set("aws", "") is None
