"""HCL2 parser/evaluator on the configurations the reference documents."""
import os

import pytest

from terraform_provider_iterative_amd.hcl import (Configuration, Context, HCLSyntaxError, parse,
                                                  parse_expression)

README_EXAMPLE = r'''
terraform {
  required_providers { iterative = { source = "iterative/iterative" } }
}
provider "iterative" {}

resource "iterative_task" "example" {
  cloud      = "aws" # or any of: gcp, az, k8s
  machine    = "m"   # medium. Or any of: l, xl, m+k80, xl+v100, ...
  spot       = 0     # auto-price. Default -1 to disable, or >0 for hourly USD limit
  disk_size  = -1    # GB. Default -1 for automatic

  storage {
    workdir = "."       # default blank (don't upload)
    output  = "results" # default blank (don't download). Relative to workdir
  }
  script = <<-END
    #!/bin/bash

    # create output directory if needed
    mkdir -p results
    # read last result (in case of spot/preemptible instance recovery)
    if test -f results/epoch.txt; then EPOCH="$(cat results/epoch.txt)"; fi
    EPOCH=$${EPOCH:-1}  # start from 1 if last result not found

    echo "(re)starting training loop from $EPOCH up to 1337 epochs"
    for epoch in $(seq $EPOCH 1337); do
      sleep 1
      echo "$epoch" | tee results/epoch.txt
    done
  END
}
'''


def test_readme_example():
    body = parse(README_EXAMPLE)
    assert [b.type for b in body.blocks] == ["terraform", "provider", "resource"]
    res = body.blocks[2]
    assert res.labels == ["iterative_task", "example"]
    ctx = Context()
    values = ctx.eval_body(res.body)
    assert values["cloud"] == "aws" and values["spot"] == 0 and values["disk_size"] == -1
    assert values["storage"] == [{"workdir": ".", "output": "results"}]
    script = values["script"]
    assert script.startswith("#!/bin/bash\n\n# create output directory if needed\n")
    assert 'EPOCH=${EPOCH:-1}  # start from 1' in script  # $${ escape
    assert script.endswith("done\n")
    req = ctx.eval_body(body.blocks[0].body)
    assert req["required_providers"][0]["iterative"]["source"] == "iterative/iterative"


def test_expressions():
    ctx = Context(variables={"n": 3, "name": "x"})
    ev = lambda s: ctx.eval(parse_expression(s))  # noqa: E731
    assert ev("1 + 2 * 3") == 7
    assert ev("var.n > 2 ? \"big\" : \"small\"") == "big"
    assert ev('"a-${var.name}-${var.n + 1}"') == "a-x-4"
    assert ev("[for i in [1, 2, 3] : i * 2 if i > 1]") == [4, 6]
    assert ev('{for k, v in {a = 1, b = 2} : k => v + 1}') == {"a": 2, "b": 3}
    assert ev('merge({a = 1}, {b = 2})') == {"a": 1, "b": 2}
    assert ev('join(",", ["a", "b"])') == "a,b"
    assert ev('lookup({a = "1"}, "b", "d")') == "d"
    assert ev('"\\u00e9\\n"') == "é\n"
    assert ev("!true") is False and ev("-(2)") == -2
    assert ev('{ "quoted key" = 1, bare: 2 }') == {"quoted key": 1, "bare": 2}
    # docs/resources/task.md:94-104: try(join("\n", iterative_task.example.logs), "")
    assert ev('try(join("\\n", var.missing), "")') == ""
    assert ev('try(var.n * 2, 0)') == 6
    assert ev('can(var.missing)') is False and ev('can(var.n)') is True


def test_heredoc_plain_and_comments():
    body = parse('# c\n/* block\n comment */\nx = <<EOF\n  keep indent\nEOF\ny = 2 // trailing\n')
    ctx = Context()
    assert ctx.eval_body(body) == {"x": "  keep indent\n", "y": 2}


def test_syntax_errors():
    with pytest.raises(HCLSyntaxError):
        parse('resource "a" "b" {\n x = \n')
    with pytest.raises(HCLSyntaxError):
        parse('x = "unterminated\n')


def test_configuration_variables_and_locals(tmp_path, monkeypatch):
    (tmp_path / "main.tf").write_text('''
variable "machine" {
  type    = string
  default = "m"
}
variable "envs" {
  type    = map(string)
  default = {}
}
locals {
  full = "${local.base}+mi355x"
  base = var.machine
}
resource "iterative_task" "t" {
  cloud   = "mi355x"
  machine = local.full
  environment = var.envs
  script  = file("run.sh")
  timeouts { create = "10m" }
}
output "status" { value = iterative_task.t.status }
''')
    (tmp_path / "run.sh").write_text("#!/bin/sh\necho hi\n")
    monkeypatch.setenv("TF_VAR_envs", '{ A = "1" }')
    cfg = Configuration(str(tmp_path), var_overrides={"machine": "l"})
    (res,) = cfg.resources("iterative_")
    values = cfg.evaluate_resource(res)
    assert values["machine"] == "l+mi355x"
    assert values["environment"] == {"A": "1"}
    assert values["script"] == "#!/bin/sh\necho hi\n"
    assert "timeouts" not in values and cfg.timeouts(res) == {"create": "10m"}
    outs = cfg.outputs({"iterative_task": {"t": {"status": {"running": 1}}}})
    assert outs["status"]["value"] == {"running": 1}
    assert os.path.isabs(cfg.context.module_dir)
