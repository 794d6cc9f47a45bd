"""Reference unit-test parity: identifier (identifier_test.go), steps (steps_test.go),
variables enrichment, status reduction, logger (logger_test.go), runner readiness
(runner_test.go), analytics (analytics_test.go), shell escaping, ssh keys."""
import json
import logging
import os
import re

import pytest

from terraform_provider_iterative_amd.models.values import Variables
from terraform_provider_iterative_amd.utils import analytics
from terraform_provider_iterative_amd.utils.identifier import (
    MAXIMUM_LONG_LENGTH, SHORT_LENGTH, WrongIdentifierError, new_deterministic_identifier,
    new_random_identifier, parse_identifier)
from terraform_provider_iterative_amd.utils.logger import (TpiFormatter, format_logs,
                                                           format_status, reduce_status)
from terraform_provider_iterative_amd.utils.runner_status import has_status
from terraform_provider_iterative_amd.utils.shell import quote, quote_command
from terraform_provider_iterative_amd.utils.steps import Step, run_steps

LONG_NAME = " ".join(["Lorem ipsum dolor sit amet, consectetur adipiscing elit"] * 40)


class TestIdentifier:
    def test_stability(self):
        i = new_deterministic_identifier(LONG_NAME)
        assert i.long() == i.long() and i.short() == i.short()

    def test_consistency(self):
        i = new_deterministic_identifier("5299fe10-79e9-4c3b-b15e-036e8e60ab6c")
        parsed = parse_identifier(i.long())
        assert parsed.long() == i.long() and parsed.short() == i.short()

    def test_homogeneity(self):
        i = new_deterministic_identifier(LONG_NAME)
        assert re.match(r"^tpi-[a-z0-9-]+$", i.long())
        assert re.match(r"^[a-z0-9]+$", i.short())
        assert len(i.long()) <= MAXIMUM_LONG_LENGTH and len(i.short()) == SHORT_LENGTH

    def test_compatibility_golden_vector(self):
        i = new_deterministic_identifier("test")
        assert i.long() == "tpi-test-3z4xlzwq-3u0vweb4"
        assert i.short() == "3z4xlzwq3u0vweb4"
        assert parse_identifier(i.long()).long() == i.long()

    def test_randomness(self):
        a, b = new_random_identifier("test"), new_random_identifier("test")
        assert a.long() != b.long() and a.short() != b.short()
        assert "test" in a.long() and "test" in b.long()
        petname = new_random_identifier("")
        assert len(petname.long().split("-")) == 6  # tpi + 3 words + salt + check

    def test_prefix(self):
        i = new_deterministic_identifier("test", prefix="ipsum")
        assert i.long() == "ips-test-3z4xlzwq-3u0vweb4"
        assert i.short() == "3z4xlzwq3u0vweb4"
        assert parse_identifier(i.long()).long() == i.long()

    def test_parse_rejects_bad_checksum(self):
        with pytest.raises(WrongIdentifierError):
            parse_identifier("tpi-test-3z4xlzwq-00000000")
        with pytest.raises(WrongIdentifierError):
            parse_identifier("not an identifier")


def test_steps_order_and_stop_on_error(caplog):
    seen = []

    def boom():
        raise RuntimeError("boom")

    steps = [Step("one", lambda: seen.append(1)), Step("two", boom),
             Step("three", lambda: seen.append(3))]
    with caplog.at_level(logging.INFO, logger="tpi"):
        with pytest.raises(RuntimeError):
            run_steps(steps)
    assert seen == [1]
    assert "[1/3] one" in caplog.text and "[2/3] two" in caplog.text
    assert "[3/3]" not in caplog.text


def test_variables_enrich():
    env = {"CI": "1", "CI_JOB": "x", "GITHUB_SHA": "abc", "OTHER": "no", "HOME": "/h"}
    v = Variables({"EXPLICIT": "v", "CI": None, "CI_*": None, "GITHUB_*": None, "MISSING": None,
                   "HO?E": None})
    assert v.enrich(env) == {"EXPLICIT": "v", "CI": "1", "CI_JOB": "x", "GITHUB_SHA": "abc"}


@pytest.mark.parametrize("status,par,want", [
    ({}, 1, "queued"), ({"succeeded": 1}, 1, "succeeded"), ({"succeeded": 1}, 2, "queued"),
    ({"succeeded": 1, "failed": 1}, 1, "failed"), ({"running": 2, "failed": 1}, 2, "running"),
])
def test_status_reduction(status, par, want):
    assert reduce_status(status, par) == want


def test_logger_formats():
    assert "completed with errors" in format_status({"status": {"running": 0, "failed": 1},
                                                     "parallelism": 1})
    assert "queued" in format_status({"status": {"running": 0, "failed": 0}, "parallelism": 1})
    out = format_logs({"logs": ["a\nb\n", "c\n"]})
    assert out.count("LOG 0 >> ") == 2 and out.count("LOG 1 >> ") == 1
    rec = logging.LogRecord("tpi", logging.INFO, "", 0, "instance", None, None)
    rec.d = {"cloud": "mi355x", "machine": "m+mi355x", "region": "us-west", "spot": 0.5}
    text = TpiFormatter().format(rec)
    assert "TPI [INFO]" in text and "mi355x m+mi355x(Spot 0.500000/h) in us-west" in text
    rec2 = logging.LogRecord("tpi", logging.INFO, "", 0, "bogus", None, None)
    rec2.d = {}
    with pytest.raises(ValueError):
        TpiFormatter().format(rec2)


def test_runner_readiness():
    ready = """
        -- Logs begin at Wed 2021-01-20 00:25:37 UTC, end at Fri 2021-02-26 15:37:56 UTC. --
        Feb 26 15:37:20 ip-172-31-6-188 cml.sh[2203]: {"level":"info","time":"···","repo":"···","status":"ready"}
    """
    assert has_status(ready, "ready")
    assert not has_status(ready.replace(',"status":"ready"', ""), "ready")


def test_shell_quote_matches_shellescape():
    assert quote("") == "''"
    assert quote("safe/path-1.txt") == "safe/path-1.txt"
    assert quote("it's") == "'it'\"'\"'s'"
    assert quote_command(["echo", "a b", "$HOME"]) == "echo 'a b' '$HOME'"


def test_analytics_deterministic_group_ids():
    # vectors documented in the reference (analytics.go:374-379)
    assert analytics.deterministic("https://github.com/iterative") == \
        "dc16cd76-71b7-5afa-bf11-e85e02ee1554"
    assert analytics.deterministic("https://bitbucket.com/iterative-test") == \
        "c0b86b90-d63c-5fb0-b84d-718d8e15f8d6"


def test_analytics_user_id_migration(tmp_path):
    env = {"XDG_CONFIG_HOME": str(tmp_path)}
    old = tmp_path / "dvc" / "user_id"
    old.parent.mkdir()
    old.write_text(json.dumps({"user_id": "00000000-0000-0000-0000-000000000000"}))
    assert analytics.user_id(env) == "00000000-0000-0000-0000-000000000000"
    assert (tmp_path / "iterative" / "telemetry").exists()


def test_analytics_resource_data_and_optout(tmp_path):
    data = {"cloud": "aws", "region": "us-west", "machine": "xl", "disk_size": 30, "spot": 0.0,
            "status": {"running": 0, "failed": 0},
            "logs": ["2022-04-24 20:25:07 Started tpi-task.service.\n2022-04-24 20:26:07 hello.\n",
                     "2022-04-24 20:27:07 Started tpi-task.service.\n"]}
    rd = analytics.resource_data(data)
    assert rd["task_duration"] == 120.0 and rd["task_resumed"] is True
    assert rd["cloud_spot_auto"] is True
    spool = tmp_path / "events.jsonl"
    env = {"XDG_CONFIG_HOME": str(tmp_path), "TPI_ANALYTICS_SPOOL": str(spool)}
    body = analytics.send_event("task/apply", ValueError("secret message"), data, env)
    assert body["error"] == "ValueError" and "secret" not in json.dumps(body)
    assert body["extra"]["cloud"] == "aws" and spool.exists()
    assert analytics.send_event("task/apply", None, data, dict(env, ITERATIVE_DO_NOT_TRACK="1")) is None
    assert analytics.send_event("task/apply", None, data, {"XDG_CONFIG_HOME": str(tmp_path)}) is None


def test_ssh_keys_roundtrip_and_determinism():
    from terraform_provider_iterative_amd.utils.ssh import (DeterministicSSHKeyPair, RSAKey,
                                                            public_from_private_pem)

    k1 = DeterministicSSHKeyPair("secret", "realm", bits=1024)
    k2 = DeterministicSSHKeyPair("secret", "realm", bits=1024)
    k3 = DeterministicSSHKeyPair("secret", "other", bits=1024)
    assert k1.private_string() == k2.private_string() != k3.private_string()
    pem = k1.private_string()
    assert pem.startswith("-----BEGIN RSA PRIVATE KEY-----")
    assert public_from_private_pem(pem) == k1.public_string()
    key = RSAKey.from_pem(pem)
    msg = 123456789
    assert pow(pow(msg, key.e, key.n), key.d, key.n) == msg
    if os.path.exists("/usr/bin/ssh-keygen"):
        import subprocess
        import tempfile

        with tempfile.NamedTemporaryFile("w", delete=False) as f:
            f.write(pem)
        os.chmod(f.name, 0o600)
        out = subprocess.run(["ssh-keygen", "-y", "-f", f.name], capture_output=True, text=True)
        os.unlink(f.name)
        assert out.returncode == 0 and out.stdout.split()[1] == k1.public_string().split()[1]


def test_set_id_cml_prefix():
    # iterative/utils/helpers_test.go:9-13
    from terraform_provider_iterative_amd.utils.helpers import set_id

    data = {"name": "example"}
    assert set_id(data).startswith("cml-example-")
    assert set_id(data) == data["id"]  # an existing id is kept


def test_helpers_cml_snippet_and_env_lookup():
    from terraform_provider_iterative_amd.utils.helpers import get_cml, multi_env_load_first

    assert get_cml().endswith("npm install --global @dvcorg/cml")
    assert get_cml("v0.18.1").endswith("@dvcorg/cml@v0.18.1")
    assert get_cml("0.18.1").endswith("@dvcorg/cml@v0.18.1")
    assert get_cml("github:iterative/cml#main").endswith("--global github:iterative/cml#main")
    env = {"A": "", "B": "b", "C": "c"}
    assert multi_env_load_first(["A", "B", "C"], env) == "b"
    assert multi_env_load_first(["X"], env) == ""


def test_cloud_descriptor():
    import pytest

    from terraform_provider_iterative_amd.models.cloud import (Cloud, Credentials,
                                                               NodeCredentials,
                                                               default_state_root,
                                                               parse_region_selectors)

    cloud = Cloud(provider="aws", region="us-east-1")
    assert cloud.get_closest_region({"us-east": "us-east-1", "us-west": "us-west-1"}) == "us-east"
    with pytest.raises(KeyError):
        cloud.get_closest_region({"eu-west": "eu-west-1"})
    assert cloud.timeouts.create == 900 and cloud.timeouts.read == 180
    assert default_state_root({"TPI_STATE_ROOT": "/x"}) == "/x"
    assert default_state_root({"HOME": "/h"}) == "/h/.local/state/tpi"
    node = Cloud(credentials=Credentials(node=NodeCredentials("/srv/tpi")))
    assert node.state_root() == "/srv/tpi"
    assert parse_region_selectors("gpus=2-3, numa=1,us-west") == {"gpus": "2-3", "numa": "1"}


def test_record_matches_dataclass_semantics():
    """utils/record.py: the dataclass subset the CLI-path value types rely on."""
    import pytest as _pytest

    from terraform_provider_iterative_amd.utils.record import (FrozenInstanceError, field,
                                                                record, replace)

    @record
    class Point:
        x: int
        y: int = 2
        tags: list = field(default_factory=list)

    a, b = Point(1), Point(1)
    assert (a.x, a.y, a.tags) == (1, 2, [])
    assert a == b and a.tags is not b.tags
    assert Point(1, 3, ["t"]) == Point(x=1, y=3, tags=["t"])
    assert repr(Point(1)).endswith("Point(x=1, y=2, tags=[])")  # __qualname__, as dataclasses
    assert replace(a, y=5) == Point(1, 5)
    with _pytest.raises(TypeError):
        Point()
    with _pytest.raises(TypeError):
        Point(1, z=3)
    with _pytest.raises(TypeError):
        Point(1, x=1)
    with _pytest.raises(TypeError):
        hash(a)

    @record(frozen=True)
    class Key:
        name: str
        n: int = 0

    k = Key("a")
    assert hash(k) == hash(Key("a")) and {k: 1}[Key("a")] == 1
    with _pytest.raises(FrozenInstanceError):
        k.n = 3
