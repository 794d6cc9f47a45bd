"""``leo``: command-line task management (reference: ``cmd/leo/**``).

    leo --cloud mi355x create [--machine m+mi355x] [--workdir .] [--output results] -- cmd...
    leo --cloud mi355x read [--follow] [--timestamps] ID
    leo --cloud mi355x list | delete ID | stop ID (hidden) | destroy-runner ID (hidden)
    leo --cloud mi355x preempt ID   (hidden; fault injection: SIGTERM the ranks, respawn)

Flag defaults come from ``./main.tf`` (the first ``iterative_task``; options ``cloud image log
machine name parallelism permission_set region script spot disk_size timeout tags environment
storage.{output,workdir,exclude}``) and ``TASK_*`` environment variables, exactly like the
reference's viper wiring (root.go:73-164); explicit flags win.  Unlike the reference (which
hard-codes 1, create.go:102) ``--parallelism`` is honoured.
"""
from __future__ import annotations

import argparse
import logging
import os
import sys
import time
from typing import Any, Dict, List, Optional

from .. import backends
from .._version import __version__
from ..hcl import Configuration
from ..models.cloud import Cloud, Credentials, NodeCredentials, Timeouts
from ..models.values import (SPOT_DISABLED, SPOT_ENABLED, Environment, Firewall, FirewallRule,
                             Size, Task as TaskSpec, Variables)
from ..utils.identifier import new_random_identifier, parse_identifier
from ..utils.logger import reduce_status, setup as setup_logging
from ..utils.shell import quote_command
from ..utils.watch import DirectoryWatch

log = logging.getLogger("tpi")

TASK_OPTIONS = ("cloud", "image", "log", "machine", "name", "parallelism", "permission_set",
                "region", "script", "spot", "disk_size", "timeout")


def config_defaults(directory: str = ".", environ=None) -> Dict[str, Any]:
    """Flag defaults from ``main.tf`` and ``TASK_*`` (``root.go:73-143``)."""
    environ = os.environ if environ is None else environ
    out: Dict[str, Any] = {}
    if os.path.exists(os.path.join(directory, "main.tf")):
        try:
            cfg = Configuration(directory, files=[os.path.join(directory, "main.tf")])
            for block in cfg.resources("iterative_task"):
                values = cfg.evaluate_resource(block)
                for option in TASK_OPTIONS:
                    if option in values:
                        out[option.replace("_", "-")] = values[option]
                for option in ("tags", "environment"):
                    if isinstance(values.get(option), dict):
                        out[option] = values[option]
                for block_values in values.get("storage") or []:
                    for key in ("output", "workdir", "exclude"):
                        if key in block_values:
                            out[key] = block_values[key]
        except Exception as error:
            log.error("error reading configuration from main.tf: %s", error)
    for key, value in environ.items():
        if key.startswith("TASK_") and len(key) > 5:
            out[key[5:].lower().replace("_", "-")] = value
    return out


class KeyValue(argparse.Action):
    """pflag StringToString: ``--environment A=1,B=2`` (repeatable)."""

    def __call__(self, parser, namespace, values, option_string=None):
        current = dict(getattr(namespace, self.dest) or {})
        for item in values.split(","):
            if not item:
                continue
            key, sep, value = item.partition("=")
            if not sep:
                parser.error("%s expects key=value pairs, got %r" % (option_string, item))
            current[key] = value
        setattr(namespace, self.dest, current)


class CommaList(argparse.Action):
    """pflag StringSlice: ``--exclude a,b`` (repeatable)."""

    def __call__(self, parser, namespace, values, option_string=None):
        current = list(getattr(namespace, self.dest) or [])
        current.extend(v for v in values.split(",") if v)
        setattr(namespace, self.dest, current)


def build_parser(defaults: Dict[str, Any]) -> argparse.ArgumentParser:
    d = defaults.get
    root = argparse.ArgumentParser(prog="leo", description="leo is a command-line tool that "
                                   "allows data scientists to run code on MI355X nodes.")
    root.add_argument("--cloud", default=d("cloud"), help="cloud provider (local, mi355x)")
    root.add_argument("--region", default=d("region", "us-east"), help="cloud region")
    root.add_argument("--verbose", action="store_true", help="verbose output")
    root.add_argument("--state-root", default=None, help="node runtime state directory")
    root.add_argument("--version", action="version", version="leo version " + __version__)
    sub = root.add_subparsers(dest="command", required=True)

    create = sub.add_parser("create", help="Create a task")
    create.add_argument("--environment", action=KeyValue, default=dict(d("environment") or {}))
    create.add_argument("--image", default=d("image", "ubuntu"))
    create.add_argument("--machine", default=d("machine", "m"))
    create.add_argument("--name", default=d("name", ""))
    create.add_argument("--output", default=d("output", ""))
    create.add_argument("--exclude", action=CommaList, default=list(d("exclude") or []))
    create.add_argument("--parallelism", type=int, default=int(d("parallelism", 1)))
    create.add_argument("--permission-set", default=d("permission-set", ""))
    create.add_argument("--script", default=d("script", ""))
    # pflag bool parsing of the config value (strconv.ParseBool)
    create.add_argument("--spot", action="store_true",
                        default=str(d("spot", "false")).lower() in ("1", "t", "true"))
    create.add_argument("--disk-size", type=int, default=int(d("disk-size", -1)))
    create.add_argument("--tags", action=KeyValue, default=dict(d("tags") or {}))
    create.add_argument("--timeout", type=int, default=int(d("timeout", 24 * 60 * 60)))
    create.add_argument("--workdir", default=d("workdir", "."))
    create.add_argument("args", nargs=argparse.REMAINDER)

    read = sub.add_parser("read", help="Read information from an existing task")
    read.add_argument("--parallelism", type=int, default=1)
    read.add_argument("--timestamps", action="store_true")
    read.add_argument("--follow", action="store_true")
    read.add_argument("name")

    sub.add_parser("list", help="List tasks")
    delete = sub.add_parser("delete", help="Delete a task")
    delete.add_argument("--output", default=d("output", ""))
    delete.add_argument("--workdir", default=d("workdir", "."))
    delete.add_argument("name")
    stop = sub.add_parser("stop", help=argparse.SUPPRESS)
    stop.add_argument("name")
    destroy_runner = sub.add_parser("destroy-runner", help=argparse.SUPPRESS)
    destroy_runner.add_argument("name")
    preempt = sub.add_parser("preempt", help=argparse.SUPPRESS)
    preempt.add_argument("name")
    preempt.add_argument("--rank", type=int, default=None,
                         help="preempt only this rank (its gang follows when coupled)")
    events = sub.add_parser("events", help=argparse.SUPPRESS)
    events.add_argument("name")
    events.add_argument("--since", default=None, metavar="CODE",
                        help="times relative to the first event with this code (e.g. "
                             "preempt-signal); default: the task's first event")
    events.add_argument("--json", action="store_true", help="one JSON object per event")
    checkpoint = sub.add_parser("checkpoint", help=argparse.SUPPRESS)
    checkpoint.add_argument("path")
    checkpoint.add_argument("--verify", action="store_true",
                            help="decode and CRC-check every tile")
    return root


def cmd_checkpoint(args) -> int:
    """Summary (and with ``--verify`` an integrity check) of a persisted checkpoint file."""
    import json

    from ..checkpoint import describe_checkpoint, verify_checkpoint

    info = describe_checkpoint(args.path)
    summary = {k: info.get(k) for k in ("format", "complete", "codec", "total", "stream_bytes",
                                         "ntiles", "tile_bytes", "ntensors", "saved_at",
                                         "saves", "metadata")}
    if info.get("total"):
        summary["ratio"] = round(int(info["stream_bytes"]) / int(info["total"]), 4)
    if args.verify:
        summary["verify"] = verify_checkpoint(args.path)
    print(json.dumps(summary, indent=1, sort_keys=True))
    ok = not args.verify or (summary["verify"].get("bad_tiles") == 0)
    return 0 if info.get("complete") and ok else 1


def _cloud(args) -> Cloud:
    if not args.cloud:
        raise SystemExit('Error: required flag(s) "cloud" not set')
    creds = Credentials(node=NodeCredentials(state_root=args.state_root or ""))
    return Cloud(provider=args.cloud, region=args.region, timeouts=Timeouts(), credentials=creds)


def cmd_create(args, cloud: Cloud) -> int:
    variables = Variables()
    for name, value in args.environment.items():
        variables[name.upper()] = value if value != "" else None
    cloud.tags = dict(args.tags)
    script = args.script
    if not script.startswith("#!"):
        script = "#!/bin/sh\n" + script
    command = list(args.args)
    if command and command[0] == "--":
        command = command[1:]
    script += "\n" + quote_command(command)
    spec = TaskSpec(size=Size(machine=args.machine, storage=args.disk_size),
                    environment=Environment(image=args.image, script=script, variables=variables,
                                            directory=args.workdir, directory_out=args.output,
                                            exclude_list=list(args.exclude),
                                            timeout=float(args.timeout)),
                    firewall=Firewall(ingress=FirewallRule(ports=[22])),
                    parallelism=max(1, args.parallelism), permission_set=args.permission_set,
                    spot=SPOT_ENABLED if args.spot else SPOT_DISABLED)
    try:
        ident = parse_identifier(args.name)
    except ValueError:
        ident = new_random_identifier(args.name)
    task = backends.new(cloud, ident, spec)
    log.info("Using identifier %s", ident.long())
    try:
        task.create()
    except Exception as error:
        log.error("Failed to create a new task: %s", error)
        log.warning("Attempting to delete residual resources...")
        try:
            task.delete()
        except Exception:
            log.error("Failed to delete residual resources")
        print(ident.long())
        return 1
    print(ident.long())
    return 0


def _log_lines(logs: List[str], timestamps: bool) -> List[str]:
    out = []
    for entry in logs:
        for line in entry.strip("\n").split("\n"):
            if not timestamps:
                _, _, line = line.partition(" ")
            out.append(line)
    return out


def cmd_read(args, cloud: Cloud, poll: float = 3.0) -> int:
    ident = parse_identifier(args.name)
    task = backends.new(cloud, ident, TaskSpec(environment=Environment(image="ubuntu")))
    # node tasks: wake up on writes to the reports/supervisor directories (inotify) rather
    # than sleeping the full poll interval
    watch_dirs = [getattr(task, "reports_dir", None), getattr(task, "sup_dir", None)]
    watch = DirectoryWatch([d for d in watch_dirs if d]) if args.follow else None
    try:
        return _read_loop(args, task, watch, poll)
    finally:
        if watch is not None:
            watch.close()


def _read_loop(args, task, watch, poll: float) -> int:
    last = 0
    first = True
    waiting = False
    while True:
        task.read()
        lines = _log_lines(task.logs(), args.timestamps)
        if first and not lines:
            sys.stderr.write("Waiting for instance")
            waiting = True
        first = False
        if waiting:
            sys.stderr.write(".")
            sys.stderr.flush()
        for event in task.events():
            line = "%s: %s" % (event.code, " ".join(event.description))
            if args.timestamps:
                line = "%s %s" % (event.time.strftime("%Y-%m-%dT%H:%M:%SZ"), line)
            log.debug(line)
        status = reduce_status(task.status(), args.parallelism)
        log.debug(status)
        delta = "\n".join(lines[last:])
        if delta:
            if waiting:
                sys.stderr.write("\n")
                waiting = False
            print(delta, flush=True)
            last = len(lines)
        if not args.follow:
            return 0
        logging.getLogger("tpi").setLevel(logging.WARNING)
        if status == "succeeded":
            return 0
        if status == "failed":
            return 1
        if watch is not None:
            watch.wait(poll)
        else:
            time.sleep(poll)


def cmd_list(args, cloud: Cloud) -> int:
    for ident in backends.list_tasks(cloud):
        print(ident.long())
    return 0


def cmd_delete(args, cloud: Cloud) -> int:
    spec = TaskSpec(environment=Environment(directory=args.workdir, directory_out=args.output))
    backends.new(cloud, parse_identifier(args.name), spec).delete()
    return 0


def cmd_stop(args, cloud: Cloud) -> int:
    backends.new(cloud, parse_identifier(args.name), TaskSpec()).stop()
    return 0


def cmd_preempt(args, cloud: Cloud) -> int:
    task = backends.new(cloud, parse_identifier(args.name), TaskSpec())
    if not hasattr(task, "preempt"):
        raise SystemExit("Error: provider %s cannot inject preemptions" % cloud.provider)
    if args.rank is None:
        task.preempt()
    else:
        task.preempt(rank=args.rank)
    return 0


def cmd_events(args, cloud: Cloud) -> int:
    """The task's phase journal (``supervisor/events.jsonl``: placement, rank starts, first
    output, preemption phases, hand-offs, exits) as a timeline in seconds."""
    import json

    task = backends.new(cloud, parse_identifier(args.name), TaskSpec())
    events = task.events()

    def seconds(event) -> float:
        t = event.time
        return t.timestamp() if hasattr(t, "timestamp") else float(t)

    if not events:
        sys.stderr.write("Error: no events for %s\n" % args.name)
        return 1
    origin = seconds(events[0])
    if args.since:
        marks = [seconds(e) for e in events if e.code == args.since]
        if not marks:
            sys.stderr.write("Error: no %s event\n" % args.since)
            return 1
        origin = marks[0]
    for event in events:
        dt = seconds(event) - origin
        if args.json:
            print(json.dumps({"t": round(dt, 4), "code": event.code,
                              "description": list(event.description)}))
        else:
            print("%+10.4f s  %-28s %s" % (dt, event.code, " | ".join(event.description)))
    return 0


def cmd_destroy_runner(args, cloud: Cloud) -> int:
    from ..provider.resources import machine_delete

    result = machine_delete({"id": args.name, "cloud": cloud.provider, "region": cloud.region})
    for diag in result.diagnostics:
        sys.stderr.write("Error: %s\n" % diag.summary)
    return 0 if result.ok else 1


COMMANDS = {"create": cmd_create, "read": cmd_read, "list": cmd_list, "delete": cmd_delete,
            "stop": cmd_stop, "destroy-runner": cmd_destroy_runner, "preempt": cmd_preempt,
            "events": cmd_events}


def main(argv: Optional[List[str]] = None) -> int:
    parser = build_parser(config_defaults("."))
    args = parser.parse_args(argv)
    setup_logging(verbose=args.verbose)
    try:
        if args.command == "checkpoint":  # file inspection: no cloud involved
            return cmd_checkpoint(args)
        return COMMANDS[args.command](args, _cloud(args))
    except SystemExit:
        raise
    except Exception as error:
        log.error("%s", error)
        return 1


if __name__ == "__main__":
    sys.exit(main())
