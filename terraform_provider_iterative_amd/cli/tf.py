"""``tpi``: a Terraform-compatible plan/apply engine for this provider's resources.

``terraform`` itself is not available on MI355X nodes of this environment, so ``tpi`` reads
``*.tf`` files (:mod:`..hcl`), diffs them against ``terraform.tfstate`` (v4, same file
Terraform would write) and drives the resource implementations directly:

    tpi init | validate | plan | apply [-auto-approve] | refresh | destroy [-auto-approve]
        | show [-json] | output [-json|-raw] [NAME] | state list|show|rm ADDR

Semantics follow Terraform + the SDK: ForceNew attribute changes replace the resource
(destroy-before-create), other changes update in place (``UpdateContext = Read`` for
``iterative_task``, resource_task.go:34), creation failures leave no state, ``-target``,
``-var``, ``-var-file``, ``TF_VAR_*``, ``-parallelism`` and ``count`` are supported.
The real Terraform plugin protocol is served by ``terraform-provider-iterative`` (see
``provider/server.py``) for sites that do have ``terraform``.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
import threading
import time
from typing import Any, Dict, List, Optional, Tuple

from ..utils.record import field, record
from ..hcl import Configuration, EvaluationError, HCLSyntaxError
from ..hcl.evaluate import Context
from ..models.schema import SchemaError, get_schema, force_new_changes, in_place_changes
from ..models.schema import normalize, parse_duration
from ..provider import resources
from ..provider.state import State, StateError, address, parse_address
from ..utils import analytics
from ..utils.logger import TpiFormatter, setup as setup_logging

SUPPORTED_PREFIX = "iterative_"


@record
class Desired:
    type: str
    name: str
    index: Any
    attrs: Dict[str, Any]
    timeouts: Dict[str, float] = field(default_factory=dict)

    @property
    def addr(self) -> str:
        return address(self.type, self.name, self.index)


@record
class Change:
    action: str  # create | delete | replace | update | noop
    type: str
    name: str
    index: Any
    before: Optional[Dict[str, Any]]
    after: Optional[Dict[str, Any]]
    reasons: List[str] = field(default_factory=list)
    timeouts: Dict[str, float] = field(default_factory=dict)

    @property
    def addr(self) -> str:
        return address(self.type, self.name, self.index)


class Engine:
    def __init__(self, directory: str = ".", state_path: Optional[str] = None,
                 var_overrides: Optional[Dict[str, str]] = None,
                 targets: Optional[List[str]] = None, parallelism: int = 10,
                 out=None, err=None):
        self.directory = os.path.abspath(directory)
        self.state_path = state_path or os.path.join(self.directory, "terraform.tfstate")
        self.var_overrides = var_overrides or {}
        self.targets = targets or []
        self.parallelism = max(1, parallelism)
        self.out = out or sys.stdout
        self.err = err or sys.stderr
        self._lock = threading.Lock()
        self._config: Optional[Configuration] = None

    # -- configuration --------------------------------------------------------------------------
    @property
    def config(self) -> Configuration:
        if self._config is None:
            self._config = Configuration(self.directory, self.var_overrides)
        return self._config

    def desired(self) -> List[Desired]:
        out = []
        for block in self.config.resources():
            type_, name = block.labels
            if not type_.startswith(SUPPORTED_PREFIX):
                continue
            count_attr = block.body.attribute("count")
            indexes: List[Any] = [None]
            if count_attr is not None:
                indexes = list(range(int(self.config.context.eval(count_attr.expr))))
            for index in indexes:
                ctx: Context = self.config.context
                ctx.scopes.append({"count": {"index": index}} if index is not None else {})
                try:
                    values = self.config.evaluate_resource(block)
                finally:
                    ctx.scopes.pop()
                values.pop("count", None)
                values.pop("depends_on", None)
                attrs = normalize(type_, values)
                timeouts = {k: parse_duration(v) for k, v in self.config.timeouts(block).items()}
                out.append(Desired(type_, name, index, attrs, timeouts))
        return out

    def _targeted(self, addr: str) -> bool:
        if not self.targets:
            return True
        return any(addr == t or addr.startswith(t + "[") for t in self.targets)

    # -- planning -------------------------------------------------------------------------------
    def plan(self, state: State, destroy: bool = False) -> List[Change]:
        changes: List[Change] = []
        wanted = {} if destroy else {d.addr: d for d in self.desired()}
        existing = {address(t, n, i): (t, n, i, inst) for t, n, i, inst in state.instances()}
        for addr, d in wanted.items():
            if not self._targeted(addr):
                continue
            if addr not in existing:
                changes.append(Change("create", d.type, d.name, d.index, None, d.attrs,
                                      timeouts=d.timeouts))
                continue
            before = existing[addr][3]["attributes"]
            replace = force_new_changes(d.type, before, d.attrs)
            if replace:
                changes.append(Change("replace", d.type, d.name, d.index, before, d.attrs,
                                      replace, d.timeouts))
            elif in_place_changes(d.type, before, d.attrs):
                changes.append(Change("update", d.type, d.name, d.index, before, d.attrs,
                                      in_place_changes(d.type, before, d.attrs), d.timeouts))
        for addr, (t, n, i, inst) in existing.items():
            if addr not in wanted and self._targeted(addr):
                changes.append(Change("delete", t, n, i, inst["attributes"], None))
        return changes

    # -- execution ------------------------------------------------------------------------------
    def _save(self, state: State) -> None:
        with self._lock:
            state.save(self.state_path)

    def _print(self, text: str, err: bool = False) -> None:
        with self._lock:
            stream = self.err if err else self.out
            stream.write(text + "\n")
            stream.flush()

    def _diagnostics(self, result: resources.Result) -> bool:
        ok = True
        for d in result.diagnostics:
            self._print("%s: %s%s" % ("Error" if d.severity == "error" else "Warning", d.summary,
                                      ("\n\n" + d.detail) if d.detail else ""),
                        err=d.severity == "error")
            ok = ok and d.severity != "error"
        return ok

    def _sensitive(self, type_: str) -> List[str]:
        return [k for k, a in get_schema(type_).attributes.items() if a.sensitive]

    def _create(self, change: Change, state: State) -> bool:
        self._print("%s: Creating..." % change.addr)
        t0 = time.time()
        result = resources.handler(change.type, "create")(dict(change.after), change.timeouts)
        ok = self._diagnostics(result)
        if result.id:
            attrs = dict(result.state)
            attrs["id"] = result.id
            with self._lock:
                state.put(change.type, change.name, attrs, change.index, change.timeouts,
                          self._sensitive(change.type))
            self._save(state)
        if ok and result.id:
            self._print("%s: Creation complete after %ds [id=%s]" % (
                change.addr, int(time.time() - t0), result.id))
        return ok and bool(result.id)

    def _delete(self, change: Change, state: State) -> bool:
        attrs = dict(change.before or {})
        self._print("%s: Destroying... [id=%s]" % (change.addr, attrs.get("id", "")))
        t0 = time.time()
        timeouts = change.timeouts
        inst = state.get(change.type, change.name, change.index)
        if inst is not None and not timeouts:
            from ..provider.state import decode_private

            timeouts = decode_private(inst.get("private", ""))
        result = resources.handler(change.type, "delete")(attrs, timeouts)
        ok = self._diagnostics(result)
        if ok:
            with self._lock:
                state.remove(change.type, change.name, change.index)
            self._save(state)
            self._print("%s: Destruction complete after %ds" % (change.addr, int(time.time() - t0)))
        return ok

    def _update(self, change: Change, state: State) -> bool:
        self._print("%s: Modifying... [id=%s]" % (change.addr, change.before.get("id", "")))
        attrs = dict(change.after)
        attrs["id"] = change.before.get("id", "")
        for key in ("ssh_public_key", "ssh_private_key", "addresses", "status", "events", "logs",
                    "instance_ip", "instance_launch_time", "ssh_public"):
            if key in change.before and key not in attrs:
                attrs[key] = change.before[key]
        result = resources.handler(change.type, "read")(attrs, change.timeouts)
        ok = self._diagnostics(result)
        with self._lock:
            state.put(change.type, change.name, result.state, change.index, change.timeouts,
                      self._sensitive(change.type))
        self._save(state)
        self._print("%s: Modifications complete [id=%s]" % (change.addr, attrs["id"]))
        return ok

    def _run_parallel(self, fn, changes: List[Change], state: State) -> List[bool]:
        if not changes:
            return []
        if len(changes) == 1 or self.parallelism <= 1:
            # one resource (the usual apply): no pool -- and no concurrent.futures import,
            # ~3 ms of every `tpi apply` start
            return [fn(c, state) for c in changes]
        from concurrent.futures import ThreadPoolExecutor

        with ThreadPoolExecutor(max_workers=self.parallelism) as pool:
            return list(pool.map(lambda c: fn(c, state), changes))

    def apply(self, changes: List[Change], state: State) -> Tuple[int, int, int, bool]:
        deletes = [c for c in changes if c.action in ("delete", "replace")]
        deleted = self._run_parallel(self._delete, deletes, state)
        ok = all(deleted)
        destroyed = sum(deleted)
        added = changed = 0
        if ok:
            creates = [c for c in changes if c.action in ("create", "replace")]
            results = self._run_parallel(self._create, creates, state)
            added = sum(results)
            ok = all(results)
            updates = [c for c in changes if c.action == "update"]
            up = self._run_parallel(self._update, updates, state)
            changed = sum(up)
            ok = ok and all(up)
        return added, changed, destroyed, ok

    def refresh(self, state: State, verbose: bool = False) -> bool:
        ok = True
        for type_, name, index, inst in list(state.instances()):
            addr = address(type_, name, index)
            if not self._targeted(addr):
                continue
            attrs = inst["attributes"]
            self._print("%s: Refreshing state... [id=%s]" % (addr, attrs.get("id", "")))
            from ..provider.state import decode_private

            result = resources.handler(type_, "read")(dict(attrs),
                                                      decode_private(inst.get("private", "")))
            ok = self._diagnostics(result) and ok
            with self._lock:
                state.put(type_, name, result.state, index, decode_private(inst.get("private", "")),
                          self._sensitive(type_))
            if verbose and type_ == "iterative_task":
                self._log_task(result.state)
        self._save(state)
        return ok

    def _log_task(self, data: Dict[str, Any]) -> None:
        formatter = TpiFormatter()
        for message in ("instance", "logs", "status"):
            record = logging.LogRecord("tpi", logging.INFO, "", 0, message, None, None)
            record.d = data
            self._print(formatter.format(record), err=True)

    def outputs(self, state: State) -> Dict[str, Any]:
        outs = self.config.outputs(state.attribute_tree())
        state.data["outputs"] = {k: {"value": v["value"], "type": _tf_type(v["value"]),
                                     **({"sensitive": True} if v["sensitive"] else {})}
                                 for k, v in outs.items()}
        return state.data["outputs"]


def _tf_type(value: Any) -> Any:
    if isinstance(value, bool):
        return "bool"
    if isinstance(value, (int, float)):
        return "number"
    if isinstance(value, str):
        return "string"
    if isinstance(value, list):
        return ["tuple", [_tf_type(v) for v in value]]
    if isinstance(value, dict):
        return ["object", {k: _tf_type(v) for k, v in value.items()}]
    return "dynamic"


# ---- rendering -----------------------------------------------------------------------------------

_SYMBOL = {"create": "+", "delete": "-", "replace": "-/+", "update": "~"}
_VERB = {"create": "will be created", "delete": "will be destroyed",
         "replace": "must be replaced", "update": "will be updated in-place"}


def _render_value(value: Any, sensitive: bool) -> str:
    if sensitive:
        return "(sensitive value)"
    if value is None:
        return "(known after apply)"
    if isinstance(value, str) and "\n" in value:
        return "<<-EOT\n" + "\n".join("            " + l for l in value.rstrip("\n").split("\n")) + \
            "\n        EOT"
    return json.dumps(value)


def render_plan(changes: List[Change]) -> str:
    lines = []
    for c in changes:
        lines.append("  # %s %s" % (c.addr, _VERB[c.action]))
        if c.reasons and c.action == "replace":
            lines.append("  # (forces replacement: %s)" % ", ".join(c.reasons))
        lines.append("  %s resource \"%s\" \"%s\" {" % (_SYMBOL[c.action], c.type, c.name))
        schema = get_schema(c.type)
        shown = c.after if c.after is not None else c.before
        for key in sorted(shown or {}):
            attr = schema.attributes.get(key)
            if attr is None or (c.action == "update" and key.split(".")[0] not in
                                [r.split(".")[0] for r in c.reasons]):
                continue
            lines.append("      %s %s = %s" % (_SYMBOL[c.action][-1], key,
                                                _render_value(shown[key], attr.sensitive)))
        lines.append("    }")
        lines.append("")
    counts = {a: sum(1 for c in changes if c.action == a) for a in _SYMBOL}
    lines.append("Plan: %d to add, %d to change, %d to destroy." % (
        counts["create"] + counts["replace"], counts["update"],
        counts["delete"] + counts["replace"]))
    return "\n".join(lines)


# ---- command line --------------------------------------------------------------------------------

def _parse_vars(args) -> Dict[str, str]:
    out: Dict[str, str] = {}
    for path in args.var_file or []:
        from ..hcl import parse_file

        ctx = Context(os.path.dirname(os.path.abspath(path)))
        for k, v in ctx.eval_body(parse_file(path)).items():
            out[k] = json.dumps(v) if not isinstance(v, str) else v
    for item in args.var or []:
        key, sep, value = item.partition("=")
        if not sep:
            raise SystemExit("Error: -var expects NAME=VALUE, got %r" % item)
        out[key] = value
    return out


def _confirm(prompt: str, auto: bool) -> bool:
    if auto:
        return True
    sys.stdout.write(prompt + "\n  Only 'yes' will be accepted to approve.\n\n  Enter a value: ")
    sys.stdout.flush()
    return sys.stdin.readline().strip() == "yes"


COMMANDS = ("init", "validate", "plan", "apply", "destroy", "refresh", "show", "output",
            "state", "version")


def _command_in(argv: List[str]) -> Optional[str]:
    """The subcommand ``argv`` names (the first word that is no option or ``-chdir``'s value)."""
    it = iter(argv)
    for tok in it:
        if tok == "-chdir":
            next(it, None)
        elif not tok.startswith("-"):
            return tok
    return None


def build_parser(only: Optional[str] = None) -> argparse.ArgumentParser:
    """The CLI's parser; ``only``: just that subcommand's parser (argparse spends ~10 ms on
    the ten of them -- gettext lookups per string -- on every ``tpi apply``)."""
    p = argparse.ArgumentParser(prog="tpi", description="Terraform-compatible engine for "
                                "iterative_* resources on the MI355X node runtime")
    p.add_argument("-chdir", dest="chdir", default=None)
    p.add_argument("-version", "--version", action="version", version=_version_text())
    sub = p.add_subparsers(dest="command", required=True)

    def common(sp, state=True, plan_opts=False):
        if state:
            sp.add_argument("-state", dest="state", default=None)
        if plan_opts:
            sp.add_argument("-var", dest="var", action="append")
            sp.add_argument("-var-file", dest="var_file", action="append")
            sp.add_argument("-target", dest="target", action="append")
            sp.add_argument("-parallelism", dest="parallelism", type=int, default=10)
            sp.add_argument("-refresh", dest="refresh", default="true")
        sp.add_argument("-no-color", dest="no_color", action="store_true")
        return sp

    def want(name: str) -> bool:
        return only is None or only == name

    if want("init"):
        common(sub.add_parser("init"), state=False)
    if want("validate"):
        common(sub.add_parser("validate"), state=False)
    if want("plan"):
        common(sub.add_parser("plan"), plan_opts=True).add_argument("-destroy",
                                                                    action="store_true")
    for name in ("apply", "destroy"):
        if want(name):
            sp = common(sub.add_parser(name), plan_opts=True)
            sp.add_argument("-auto-approve", dest="auto_approve", action="store_true")
    if want("refresh"):
        common(sub.add_parser("refresh"), plan_opts=True)
    if want("show"):
        sp = common(sub.add_parser("show"))
        sp.add_argument("-json", dest="json", action="store_true")
    if want("output"):
        sp = common(sub.add_parser("output"))
        sp.add_argument("-json", dest="json", action="store_true")
        sp.add_argument("-raw", dest="raw", action="store_true")
        sp.add_argument("name", nargs="?")
    if want("state"):
        sp = common(sub.add_parser("state"))
        sp.add_argument("subcommand", choices=("list", "show", "rm"))
        sp.add_argument("addresses", nargs="*")
    if want("version"):
        sub.add_parser("version")
    return p


def _version_text() -> str:
    from .._version import __version__

    return ("tpi v%s\non linux_amd64\n+ provider registry.terraform.io/iterative/iterative v%s"
            % (__version__, __version__))


def main(argv: Optional[List[str]] = None) -> int:
    words = sys.argv[1:] if argv is None else argv
    command = _command_in(words)
    args = build_parser(command if command in COMMANDS else None).parse_args(words)
    if args.chdir:
        os.chdir(args.chdir)
    verbose = bool(os.environ.get("TF_LOG_PROVIDER") or os.environ.get("TF_LOG"))
    setup_logging(verbose=False, formatter=TpiFormatter(),
                  level=logging.INFO if verbose else logging.WARNING)
    try:
        return _dispatch(args, verbose)
    except (HCLSyntaxError, EvaluationError, SchemaError, StateError) as error:
        sys.stderr.write("Error: %s\n" % error)
        return 1
    finally:
        analytics.wait_for_analytics()


def _dispatch(args, verbose: bool) -> int:
    cmd = args.command
    if cmd == "version":
        print(_version_text())
        return 0
    if cmd == "init":
        os.makedirs(".terraform", exist_ok=True)
        Configuration(".")
        print("Terraform has been successfully initialized! (tpi engine, provider iterative)")
        return 0
    if cmd == "validate":
        Engine(".").desired()
        print("Success! The configuration is valid.")
        return 0
    state_path = getattr(args, "state", None) or "terraform.tfstate"
    engine = Engine(".", state_path, _parse_vars(args) if hasattr(args, "var") else None,
                    getattr(args, "target", None), getattr(args, "parallelism", 10))
    if cmd in ("show", "output", "state"):
        state = State.load(state_path)
        if cmd == "show":
            if args.json:
                print(json.dumps(state.data, indent=2))
            else:
                for t, n, i, inst in state.instances():
                    print("# %s:" % address(t, n, i))
                    print(json.dumps(inst["attributes"], indent=2))
            return 0
        if cmd == "output":
            outs = state.data.get("outputs") or {}
            if args.name:
                if args.name not in outs:
                    sys.stderr.write("Error: Output %r not found\n" % args.name)
                    return 1
                value = outs[args.name]["value"]
                print(value if args.raw and isinstance(value, str) else json.dumps(value, indent=2))
            else:
                print(json.dumps(outs, indent=2) if args.json else
                      "\n".join("%s = %s" % (k, json.dumps(v["value"])) for k, v in outs.items()))
            return 0
        if args.subcommand == "list":
            print("\n".join(state.addresses()))
            return 0
        with State.locked(state_path, "OperationTypeState"):
            for addr in args.addresses:
                t, n, i = parse_address(addr)
                inst = state.get(t, n, i)
                if inst is None:
                    sys.stderr.write("Error: No instance found for %s\n" % addr)
                    return 1
                if args.subcommand == "show":
                    print(json.dumps(inst["attributes"], indent=2))
                else:
                    state.remove(t, n, i)
                    print("Removed %s" % addr)
            if args.subcommand == "rm":
                state.save(state_path)
        return 0
    with State.locked(state_path):
        state = State.load(state_path)
        if getattr(args, "refresh", "true") != "false" and state.instances():
            engine.refresh(state, verbose)
        if cmd == "refresh":
            engine.outputs(state)
            state.save(state_path)
            return 0
        destroy = cmd == "destroy" or getattr(args, "destroy", False)
        changes = engine.plan(state, destroy=destroy)
        if not changes:
            print("\nNo changes. Your infrastructure matches the configuration.")
            if cmd == "apply":
                engine.outputs(state)
                state.save(state_path)
            return 0
        print(render_plan(changes))
        if cmd == "plan":
            return 0
        verb = "destroy all remote objects" if destroy else "perform these actions"
        if not _confirm("\nDo you want to %s?" % verb, args.auto_approve):
            print("\nApply cancelled.")
            return 1
        added, changed, destroyed, ok = engine.apply(changes, state)
        if not destroy:
            engine.outputs(state)
            state.save(state_path)
        if not ok:  # like terraform: the errors above, no completion summary
            return 1
        if destroy:
            print("\nDestroy complete! Resources: %d destroyed." % destroyed)
        else:
            print("\nApply complete! Resources: %d added, %d changed, %d destroyed." % (
                added, changed, destroyed))
            for k, v in (state.data.get("outputs") or {}).items():
                print("%s = %s" % (k, "<sensitive>" if v.get("sensitive") else json.dumps(v["value"])))
        return 0


if __name__ == "__main__":
    sys.exit(main())
