"""Evaluation of parsed HCL expressions and Terraform-style configurations.

:class:`Context` resolves ``var.*`` (variable defaults, ``TF_VAR_*``, ``-var``), ``local.*``,
``path.module``/``path.root``/``path.cwd`` and ``<resource type>.<name>.<attr>`` references
(from state, for outputs), and implements the Terraform functions these configurations use.
"""
from __future__ import annotations

import base64
import json
import os
from typing import Any, Callable, Dict, List, Optional

from .parser import (Attribute, Binary, Block, Body, Call, Conditional, ForExpr, GetAttr,
                     Index, Literal, ObjectExpr, Reference, Template, TupleExpr, Unary,
                     parse_file)


def _hashlib():
    import hashlib  # lazily: ~3 ms of CLI start-up, needed only by sha256() / md5()

    return hashlib


class EvaluationError(ValueError):
    pass


class Unknown:
    """A value only known after apply (resource attributes before creation)."""

    def __repr__(self) -> str:  # pragma: no cover
        return "<unknown>"


UNKNOWN = Unknown()


def _tostring(value: Any) -> str:
    if isinstance(value, bool):
        return "true" if value else "false"
    if value is None:
        return ""
    if isinstance(value, float) and value.is_integer():
        return str(int(value))
    if isinstance(value, (dict, list)):
        raise EvaluationError("cannot interpolate a %s into a string" % type(value).__name__)
    return str(value)


def _number(value: Any):
    if isinstance(value, bool):
        raise EvaluationError("cannot use a bool as a number")
    if isinstance(value, (int, float)):
        return value
    try:
        f = float(value)
        return int(f) if f.is_integer() and "." not in str(value) else f
    except (TypeError, ValueError):
        raise EvaluationError("%r is not a number" % (value,)) from None


class Context:
    def __init__(self, module_dir: str = ".", variables: Optional[Dict[str, Any]] = None,
                 locals_: Optional[Dict[str, Any]] = None,
                 resources: Optional[Dict[str, Dict[str, Any]]] = None):
        self.module_dir = os.path.abspath(module_dir)
        self.variables = dict(variables or {})
        self.locals = dict(locals_ or {})
        self.resources = resources or {}
        self.scopes: List[Dict[str, Any]] = []
        self.functions: Dict[str, Callable[..., Any]] = self._functions()

    # -- functions -------------------------------------------------------------------------------
    def _path(self, p: str) -> str:
        return p if os.path.isabs(p) else os.path.join(self.module_dir, p)

    def _functions(self) -> Dict[str, Callable[..., Any]]:
        def file_(p):
            with open(self._path(p)) as handle:
                return handle.read()

        def filebase64(p):
            with open(self._path(p), "rb") as handle:
                return base64.b64encode(handle.read()).decode()

        def lookup(m, k, *default):
            if k in m:
                return m[k]
            if default:
                return default[0]
            raise EvaluationError("lookup: key %r not found" % k)

        def merge(*maps):
            out: Dict[str, Any] = {}
            for m in maps:
                out.update(m or {})
            return out

        def concat(*lists):
            out: List[Any] = []
            for l in lists:
                out.extend(l)
            return out

        def format_(fmt, *args):
            return fmt.replace("%%", "\0") % tuple(args) if "%" in fmt else fmt

        return {
            "file": file_, "filebase64": filebase64, "fileexists": lambda p: os.path.exists(self._path(p)),
            "abspath": os.path.abspath, "basename": os.path.basename, "dirname": os.path.dirname,
            "pathexpand": os.path.expanduser, "jsonencode": lambda v: json.dumps(v, separators=(",", ":")),
            "jsondecode": json.loads, "lower": lambda s: s.lower(), "upper": lambda s: s.upper(),
            "trimspace": lambda s: s.strip(), "chomp": lambda s: s.rstrip("\r\n"),
            "title": lambda s: s.title(), "replace": lambda s, a, b: s.replace(a, b),
            "join": lambda sep, l: sep.join(_tostring(x) for x in l), "split": lambda sep, s: s.split(sep),
            "tostring": _tostring, "tonumber": _number, "tobool": lambda v: v in (True, "true"),
            "tolist": list, "toset": lambda l: sorted(set(l), key=str), "tomap": dict,
            "concat": concat, "merge": merge, "lookup": lookup, "length": len,
            "keys": lambda m: sorted(m.keys()), "values": lambda m: [m[k] for k in sorted(m)],
            "contains": lambda l, v: v in l, "element": lambda l, i: l[int(i) % len(l)],
            "coalesce": lambda *a: next((x for x in a if x not in (None, "")), None),
            "min": min, "max": max, "abs": abs, "ceil": lambda x: -(-x // 1), "floor": lambda x: x // 1,
            "format": format_, "base64encode": lambda s: base64.b64encode(s.encode()).decode(),
            "base64decode": lambda s: base64.b64decode(s).decode(),
            "sha256": lambda s: _hashlib().sha256(s.encode()).hexdigest(),
            "md5": lambda s: _hashlib().md5(s.encode()).hexdigest(),
            "timestamp": lambda: __import__("datetime").datetime.utcnow().strftime("%Y-%m-%dT%H:%M:%SZ"),
            "__splat__": lambda v: v if isinstance(v, list) else [v],
        }

    # -- evaluation ------------------------------------------------------------------------------
    def eval(self, node: Any) -> Any:
        if isinstance(node, Literal):
            return node.value
        if isinstance(node, Template):
            if len(node.parts) == 1 and not isinstance(node.parts[0], str):
                return self.eval(node.parts[0])
            out = []
            for part in node.parts:
                if isinstance(part, str):
                    out.append(part)
                else:
                    value = self.eval(part)
                    if value is UNKNOWN:
                        return UNKNOWN
                    out.append(_tostring(value))
            return "".join(out)
        if isinstance(node, TupleExpr):
            return [self.eval(i) for i in node.items]
        if isinstance(node, ObjectExpr):
            out = {}
            for k, v in node.items:
                key = k.name if isinstance(k, Reference) else self.eval(k)
                out[_tostring(key)] = self.eval(v)
            return out
        if isinstance(node, Reference):
            return self._resolve_root(node.name)
        if isinstance(node, GetAttr):
            obj = self.eval(node.obj)
            if obj is UNKNOWN:
                return UNKNOWN
            if isinstance(obj, dict):
                if node.name not in obj:
                    raise EvaluationError("unsupported attribute %r" % node.name)
                return obj[node.name]
            raise EvaluationError("cannot access attribute %r of %r" % (node.name, obj))
        if isinstance(node, Index):
            obj, key = self.eval(node.obj), self.eval(node.key)
            if obj is UNKNOWN:
                return UNKNOWN
            if isinstance(obj, list):
                return obj[int(_number(key))]
            return obj[_tostring(key)]
        if isinstance(node, Call):
            if node.name in ("try", "can"):  # lazy: errors in an argument are the point
                for arg in node.args:
                    try:
                        value = self.eval(arg)
                    except (EvaluationError, KeyError, IndexError, TypeError, ValueError,
                            AttributeError):
                        if node.name == "can":
                            return False
                        continue
                    if value is UNKNOWN:
                        return UNKNOWN
                    return True if node.name == "can" else value
                if node.name == "can":
                    return False
                raise EvaluationError("try(): no expression succeeded")
            fn = self.functions.get(node.name)
            if fn is None:
                raise EvaluationError("unknown function %s()" % node.name)
            args = [self.eval(a) for a in node.args]
            if node.expand_final and args:
                args = args[:-1] + list(args[-1])
            return fn(*args)
        if isinstance(node, Unary):
            v = self.eval(node.operand)
            return (not v) if node.op == "!" else -_number(v)
        if isinstance(node, Binary):
            return self._binary(node)
        if isinstance(node, Conditional):
            return self.eval(node.then) if self.eval(node.cond) else self.eval(node.other)
        if isinstance(node, ForExpr):
            return self._for(node)
        raise EvaluationError("cannot evaluate %r" % (node,))

    def _binary(self, node: Binary):
        op = node.op
        if op == "&&":
            return bool(self.eval(node.left)) and bool(self.eval(node.right))
        if op == "||":
            return bool(self.eval(node.left)) or bool(self.eval(node.right))
        a, b = self.eval(node.left), self.eval(node.right)
        if op == "==":
            return a == b
        if op == "!=":
            return a != b
        a, b = _number(a), _number(b)
        return {"+": lambda: a + b, "-": lambda: a - b, "*": lambda: a * b,
                "/": lambda: a / b, "%": lambda: a % b, "<": lambda: a < b,
                ">": lambda: a > b, "<=": lambda: a <= b, ">=": lambda: a >= b}[op]()

    def _for(self, node: ForExpr):
        coll = self.eval(node.collection)
        items = list(coll.items()) if isinstance(coll, dict) else list(enumerate(coll))
        out_list, out_map = [], {}
        for k, v in items:
            scope = {node.value_var: v}
            if node.key_var:
                scope[node.key_var] = k
            self.scopes.append(scope)
            try:
                if node.cond is not None and not self.eval(node.cond):
                    continue
                if node.is_object:
                    out_map[_tostring(self.eval(node.key_expr))] = self.eval(node.value_expr)
                else:
                    out_list.append(self.eval(node.value_expr))
            finally:
                self.scopes.pop()
        return out_map if node.is_object else out_list

    def _resolve_root(self, name: str):
        for scope in reversed(self.scopes):
            if name in scope:
                return scope[name]
        if name == "var":
            return self.variables
        if name == "local":
            return self.locals
        if name == "path":
            return {"module": self.module_dir, "root": self.module_dir, "cwd": os.getcwd()}
        if name == "terraform":
            return {"workspace": os.environ.get("TF_WORKSPACE", "default")}
        if name in self.resources:
            return self.resources[name]
        raise EvaluationError("unknown reference %r" % name)

    def eval_body(self, body: Body, skip_blocks=()) -> Dict[str, Any]:
        """Attributes as a dict; nested blocks as lists of dicts keyed by block type."""
        out: Dict[str, Any] = {a.name: self.eval(a.expr) for a in body.attributes}
        for block in body.blocks:
            if block.type in skip_blocks:
                continue
            out.setdefault(block.type, []).append(self.eval_body(block.body))
        return out


def _typed_var(raw: str, decl_type: str) -> Any:
    """``-var``/``TF_VAR_`` strings are HCL for complex types, plain for strings."""
    if decl_type and not decl_type.startswith("string"):
        from .parser import parse_expression

        try:
            return Context().eval(parse_expression(raw))
        except Exception:
            return raw
    return raw


class Configuration:
    """A Terraform module directory (all ``*.tf`` files) with variables and locals resolved."""

    def __init__(self, directory: str = ".", var_overrides: Optional[Dict[str, str]] = None,
                 files: Optional[List[str]] = None, environ=None):
        environ = os.environ if environ is None else environ
        self.directory = os.path.abspath(directory)
        paths = files or sorted(os.path.join(self.directory, f) for f in os.listdir(self.directory)
                                if f.endswith(".tf"))
        self.body = Body()
        for path in paths:
            part = parse_file(path)
            self.body.attributes.extend(part.attributes)
            self.body.blocks.extend(part.blocks)
        ctx = Context(self.directory)
        variables: Dict[str, Any] = {}
        for block in self.body.blocks_of("variable"):
            name = block.labels[0]
            type_attr = block.body.attribute("type")
            decl_type = _type_name(type_attr.expr) if type_attr else ""
            default = block.body.attribute("default")
            if var_overrides and name in var_overrides:
                variables[name] = _typed_var(var_overrides[name], decl_type)
            elif "TF_VAR_" + name in environ:
                variables[name] = _typed_var(environ["TF_VAR_" + name], decl_type)
            elif default is not None:
                variables[name] = ctx.eval(default.expr)
            else:
                raise EvaluationError("no value for required variable %r" % name)
        self.variables = variables
        ctx.variables = variables
        # locals may reference each other: iterate to a fixed point
        pending: List[Attribute] = [a for b in self.body.blocks_of("locals") for a in b.body.attributes]
        for _ in range(len(pending) + 1):
            progress = []
            for attr in pending:
                try:
                    ctx.locals[attr.name] = ctx.eval(attr.expr)
                    progress.append(attr)
                except EvaluationError:
                    continue
            pending = [a for a in pending if a not in progress]
            if not pending or not progress:
                break
        if pending:
            raise EvaluationError("cannot evaluate locals: %s" % ", ".join(a.name for a in pending))
        self.context = ctx

    def resources(self, type_prefix: str = "") -> List[Block]:
        return [b for b in self.body.blocks_of("resource")
                if len(b.labels) == 2 and b.labels[0].startswith(type_prefix)]

    def evaluate_resource(self, block: Block) -> Dict[str, Any]:
        return self.context.eval_body(block.body, skip_blocks=("lifecycle", "timeouts",
                                                               "provisioner", "connection"))

    def timeouts(self, block: Block) -> Dict[str, str]:
        out: Dict[str, str] = {}
        for t in block.body.blocks_of("timeouts"):
            out.update({k: str(v) for k, v in self.context.eval_body(t.body).items()})
        return out

    def outputs(self, resources: Dict[str, Dict[str, Any]]) -> Dict[str, Any]:
        self.context.resources = resources
        out = {}
        for block in self.body.blocks_of("output"):
            attr = block.body.attribute("value")
            if attr is None:
                continue
            try:
                out[block.labels[0]] = {"value": self.context.eval(attr.expr),
                                        "sensitive": bool(self.context.eval(
                                            block.body.attribute("sensitive").expr))
                                        if block.body.attribute("sensitive") else False}
            except (EvaluationError, KeyError, IndexError):
                continue
        return out


def _type_name(expr: Any) -> str:
    if isinstance(expr, Reference):
        return expr.name
    if isinstance(expr, Call):
        return expr.name
    return ""


__all__ = ["Context", "Configuration", "EvaluationError", "UNKNOWN", "Block"]
