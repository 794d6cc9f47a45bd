"""HCL2 native-syntax parser (the subset Terraform configurations of this provider use).

Supported: blocks with labels, attributes, nested blocks, ``#``/``//``/``/* */`` comments,
numbers, booleans, ``null``, strings with ``${...}`` interpolation and ``$${``/``%%{``
escapes, heredocs (``<<EOF`` and indent-stripping ``<<-EOF``), tuples, objects (``=`` or
``:``), references with attribute/index access and splats-free traversal, function calls,
unary/binary operators and the conditional operator.

Produces an AST of :class:`Body`/:class:`Block`/:class:`Attribute` with expression nodes
that :mod:`.evaluate` turns into Python values.  ``terraform`` and ``python-hcl2`` are not
available in this environment; this parser is what ``leo`` and ``tpi`` read ``main.tf`` with
(reference: ``cmd/leo/root.go:78-143`` reads it with viper's HCL decoder).
"""
from __future__ import annotations

import re
from typing import Any, List, Optional, Tuple, Union

from ..utils.record import field, record


class HCLSyntaxError(ValueError):
    def __init__(self, message: str, line: int = 0, filename: str = ""):
        where = "%s:%d: " % (filename or "<hcl>", line) if line else ""
        super().__init__(where + message)
        self.line = line


# ---- AST -----------------------------------------------------------------------------------

@record
class Literal:
    value: Any


@record
class Template:
    parts: List[Union[str, Any]]  # str chunks and expression nodes


@record
class TupleExpr:
    items: List[Any]


@record
class ObjectExpr:
    items: List[Tuple[Any, Any]]  # (key expr, value expr)


@record
class Reference:
    name: str


@record
class GetAttr:
    obj: Any
    name: str


@record
class Index:
    obj: Any
    key: Any


@record
class Call:
    name: str
    args: List[Any]
    expand_final: bool = False


@record
class Unary:
    op: str
    operand: Any


@record
class Binary:
    op: str
    left: Any
    right: Any


@record
class Conditional:
    cond: Any
    then: Any
    other: Any


@record
class ForExpr:
    key_var: Optional[str]
    value_var: str
    collection: Any
    key_expr: Optional[Any]
    value_expr: Any
    cond: Optional[Any]
    is_object: bool


@record
class Attribute:
    name: str
    expr: Any
    line: int = 0


@record
class Block:
    type: str
    labels: List[str]
    body: "Body"
    line: int = 0


@record
class Body:
    attributes: List[Attribute] = field(default_factory=list)
    blocks: List[Block] = field(default_factory=list)

    def attribute(self, name: str) -> Optional[Attribute]:
        for attr in self.attributes:
            if attr.name == name:
                return attr
        return None

    def blocks_of(self, type_: str) -> List[Block]:
        return [b for b in self.blocks if b.type == type_]


# ---- lexer ---------------------------------------------------------------------------------

_TOKEN_RE = re.compile(r"""
    (?P<ws>[ \t\r]+)
  | (?P<comment>\#[^\n]*|//[^\n]*|/\*.*?\*/)
  | (?P<nl>\n)
  | (?P<heredoc><<-?[A-Za-z_][A-Za-z0-9_]*[ \t]*\n)
  | (?P<number>\d+(?:\.\d+)?(?:[eE][+-]?\d+)?)
  | (?P<ident>[A-Za-z_][A-Za-z0-9_-]*)
  | (?P<string>")
  | (?P<op>==|!=|<=|>=|&&|\|\||=>|\.\.\.|[-+*/%<>!?:=.,\[\](){}])
""", re.X | re.S)


@record
class Tok:
    kind: str
    value: Any
    line: int


def _scan_template(src: str, pos: int, line: int, end_char: Optional[str],
                   filename: str) -> Tuple[List[Union[str, Any]], int, int]:
    """Scan a quoted-string/heredoc template body starting at ``pos``.

    For quoted strings ``end_char`` is '"'; for heredocs it is None and the whole text is
    the template.  Returns (parts, new_pos, new_line).
    """
    parts: List[Union[str, Any]] = []
    buf: List[str] = []
    n = len(src)
    while pos < n:
        c = src[pos]
        if end_char is not None and c == end_char:
            break
        if end_char is not None and c == "\n":
            raise HCLSyntaxError("unterminated string", line, filename)
        if c == "\\" and end_char is not None:
            if pos + 1 >= n:
                raise HCLSyntaxError("bad escape", line, filename)
            e = src[pos + 1]
            mapping = {"n": "\n", "t": "\t", "r": "\r", '"': '"', "\\": "\\"}
            if e in mapping:
                buf.append(mapping[e])
                pos += 2
                continue
            if e == "u" and pos + 6 <= n:
                buf.append(chr(int(src[pos + 2:pos + 6], 16)))
                pos += 6
                continue
            if e == "U" and pos + 10 <= n:
                buf.append(chr(int(src[pos + 2:pos + 10], 16)))
                pos += 10
                continue
            raise HCLSyntaxError("invalid escape \\%s" % e, line, filename)
        if src.startswith("$${", pos) or src.startswith("%%{", pos):
            buf.append(c + "{")
            pos += 3
            continue
        if src.startswith("${", pos) or src.startswith("%{", pos):
            directive = c == "%"
            depth, j = 1, pos + 2
            in_str = False
            while j < n and depth:
                ch = src[j]
                if in_str:
                    if ch == "\\":
                        j += 1
                    elif ch == '"':
                        in_str = False
                elif ch == '"':
                    in_str = True
                elif ch == "{":
                    depth += 1
                elif ch == "}":
                    depth -= 1
                j += 1
            if depth:
                raise HCLSyntaxError("unterminated interpolation", line, filename)
            inner = src[pos + 2:j - 1]
            if buf:
                parts.append("".join(buf))
                buf = []
            if directive:
                # Template directives (%{if}/%{for}) are kept verbatim: the provider's
                # attributes never need them evaluated.
                parts.append("%{" + inner + "}")
            else:
                strip = inner.strip().lstrip("~").rstrip("~")
                parts.append(parse_expression(strip, filename, line))
            line += inner.count("\n")
            pos = j
            continue
        if c == "\n":
            line += 1
        buf.append(c)
        pos += 1
    if buf:
        parts.append("".join(buf))
    return parts, pos, line


def tokenize(src: str, filename: str = "") -> List[Tok]:
    toks: List[Tok] = []
    pos, line, n = 0, 1, len(src)
    while pos < n:
        m = _TOKEN_RE.match(src, pos)
        if not m:
            raise HCLSyntaxError("unexpected character %r" % src[pos], line, filename)
        kind = m.lastgroup
        text = m.group(kind)
        if kind == "ws":
            pos = m.end()
            continue
        if kind == "comment":
            line += text.count("\n")
            pos = m.end()
            continue
        if kind == "nl":
            toks.append(Tok("nl", "\n", line))
            line += 1
            pos = m.end()
            continue
        if kind == "string":
            parts, end, new_line = _scan_template(src, m.end(), line, '"', filename)
            if end >= n:
                raise HCLSyntaxError("unterminated string", line, filename)
            toks.append(Tok("template", parts, line))
            line = new_line
            pos = end + 1
            continue
        if kind == "heredoc":
            strip_indent = text.startswith("<<-")
            marker = text[3 if strip_indent else 2:].strip()
            body_start = m.end()
            # find the closing marker on its own line
            end_re = re.compile(r"^[ \t]*" + re.escape(marker) + r"[ \t]*$", re.M)
            em = end_re.search(src, body_start)
            if not em:
                raise HCLSyntaxError("unterminated heredoc %s" % marker, line, filename)
            body = src[body_start:em.start()]
            if strip_indent:
                lines = body.split("\n")
                content = [l for l in lines if l.strip()]
                indent = min((len(l) - len(l.lstrip(" \t")) for l in content), default=0)
                body = "\n".join(l[indent:] for l in lines)
            parts, _, _ = _scan_template(body, 0, line + 1, None, filename)
            toks.append(Tok("template", parts, line))
            line += 1 + body.count("\n")
            pos = em.end()
            continue
        if kind == "number":
            value = float(text) if any(ch in text for ch in ".eE") else int(text)
            toks.append(Tok("number", value, line))
        elif kind == "ident":
            toks.append(Tok("ident", text, line))
        else:
            toks.append(Tok("op", text, line))
        pos = m.end()
    toks.append(Tok("eof", None, line))
    return toks


# ---- parser --------------------------------------------------------------------------------

_BINARY = [("||",), ("&&",), ("==", "!="), ("<", ">", "<=", ">="), ("+", "-"), ("*", "/", "%")]


class Parser:
    def __init__(self, toks: List[Tok], filename: str = ""):
        self.toks = toks
        self.i = 0
        self.filename = filename
        self.nl_depth = 0  # >0 inside ( [ { where newlines are insignificant

    # token helpers
    def peek(self, skip_nl: bool = None) -> Tok:
        skip = self.nl_depth > 0 if skip_nl is None else skip_nl
        j = self.i
        while skip and self.toks[j].kind == "nl":
            j += 1
        return self.toks[j]

    def next(self, skip_nl: bool = None) -> Tok:
        skip = self.nl_depth > 0 if skip_nl is None else skip_nl
        while skip and self.toks[self.i].kind == "nl":
            self.i += 1
        tok = self.toks[self.i]
        self.i += 1
        return tok

    def expect_op(self, op: str, skip_nl: bool = None) -> Tok:
        tok = self.next(skip_nl)
        if tok.kind != "op" or tok.value != op:
            self.error("expected %r, got %r" % (op, tok.value), tok)
        return tok

    def error(self, message: str, tok: Optional[Tok] = None):
        raise HCLSyntaxError(message, (tok or self.peek()).line, self.filename)

    def skip_nl(self) -> None:
        while self.toks[self.i].kind == "nl":
            self.i += 1

    # structure
    def parse_body(self, closing: Optional[str]) -> Body:
        body = Body()
        while True:
            self.skip_nl()
            tok = self.peek(False)
            if tok.kind == "eof":
                if closing:
                    self.error("unexpected end of file, expected %r" % closing, tok)
                return body
            if tok.kind == "op" and tok.value == closing:
                self.next(False)
                return body
            if tok.kind != "ident":
                self.error("expected attribute or block, got %r" % (tok.value,), tok)
            name_tok = self.next(False)
            nxt = self.peek(False)
            if nxt.kind == "op" and nxt.value in ("=", ":"):
                self.next(False)
                expr = self.parse_expr()
                body.attributes.append(Attribute(name_tok.value, expr, name_tok.line))
                end = self.peek(False)
                if end.kind not in ("nl", "eof") and not (end.kind == "op" and end.value == closing):
                    self.error("expected newline after attribute %s" % name_tok.value, end)
                continue
            labels = []
            while True:
                nxt = self.peek(False)
                if nxt.kind == "template":
                    self.next(False)
                    if any(not isinstance(p, str) for p in nxt.value):
                        self.error("block labels cannot be interpolated", nxt)
                    labels.append("".join(nxt.value))
                elif nxt.kind == "ident":
                    self.next(False)
                    labels.append(nxt.value)
                else:
                    break
            self.expect_op("{", False)
            inner = self.parse_body("}")
            body.blocks.append(Block(name_tok.value, labels, inner, name_tok.line))

    # expressions
    def parse_expr(self):
        cond = self.parse_binary(0)
        tok = self.peek()
        if tok.kind == "op" and tok.value == "?":
            self.next()
            self.nl_depth += 1
            then = self.parse_expr()
            self.expect_op(":")
            other = self.parse_expr()
            self.nl_depth -= 1
            return Conditional(cond, then, other)
        return cond

    def parse_binary(self, level: int):
        if level >= len(_BINARY):
            return self.parse_unary()
        left = self.parse_binary(level + 1)
        while True:
            tok = self.peek()
            if tok.kind == "op" and tok.value in _BINARY[level]:
                self.next()
                right = self.parse_binary(level + 1)
                left = Binary(tok.value, left, right)
            else:
                return left

    def parse_unary(self):
        tok = self.peek()
        if tok.kind == "op" and tok.value in ("!", "-"):
            self.next()
            return Unary(tok.value, self.parse_unary())
        return self.parse_postfix(self.parse_primary())

    def parse_postfix(self, node):
        while True:
            tok = self.peek()
            if tok.kind == "op" and tok.value == ".":
                self.next()
                name = self.next()
                if name.kind == "ident":
                    node = GetAttr(node, name.value)
                elif name.kind == "number":
                    node = Index(node, Literal(name.value))
                elif name.kind == "op" and name.value == "*":
                    node = Call("__splat__", [node])
                else:
                    self.error("expected attribute name", name)
            elif tok.kind == "op" and tok.value == "[":
                self.next()
                self.nl_depth += 1
                key = self.parse_expr()
                self.expect_op("]")
                self.nl_depth -= 1
                node = Index(node, key)
            else:
                return node

    def parse_primary(self):
        tok = self.next()
        if tok.kind == "number":
            return Literal(tok.value)
        if tok.kind == "template":
            parts = tok.value
            if len(parts) == 1 and not isinstance(parts[0], str):
                return Template(parts)
            if all(isinstance(p, str) for p in parts):
                return Literal("".join(parts))
            return Template(parts)
        if tok.kind == "ident":
            if tok.value == "true":
                return Literal(True)
            if tok.value == "false":
                return Literal(False)
            if tok.value == "null":
                return Literal(None)
            nxt = self.peek(False)
            if nxt.kind == "op" and nxt.value == "(":
                self.next(False)
                self.nl_depth += 1
                args, expand = [], False
                while not (self.peek().kind == "op" and self.peek().value == ")"):
                    args.append(self.parse_expr())
                    t = self.peek()
                    if t.kind == "op" and t.value == "...":
                        self.next()
                        expand = True
                    if self.peek().kind == "op" and self.peek().value == ",":
                        self.next()
                self.expect_op(")")
                self.nl_depth -= 1
                return Call(tok.value, args, expand)
            return Reference(tok.value)
        if tok.kind == "op" and tok.value == "(":
            self.nl_depth += 1
            expr = self.parse_expr()
            self.expect_op(")")
            self.nl_depth -= 1
            return expr
        if tok.kind == "op" and tok.value == "[":
            self.nl_depth += 1
            if self.peek().kind == "ident" and self.peek().value == "for":
                node = self.parse_for(False)
                self.nl_depth -= 1
                return node
            items = []
            while not (self.peek().kind == "op" and self.peek().value == "]"):
                items.append(self.parse_expr())
                if self.peek().kind == "op" and self.peek().value == ",":
                    self.next()
            self.expect_op("]")
            self.nl_depth -= 1
            return TupleExpr(items)
        if tok.kind == "op" and tok.value == "{":
            self.nl_depth += 1
            if self.peek().kind == "ident" and self.peek().value == "for":
                node = self.parse_for(True)
                self.nl_depth -= 1
                return node
            items = []
            while not (self.peek().kind == "op" and self.peek().value == "}"):
                ktok = self.peek()
                if ktok.kind == "ident" and self.toks[self._next_index()].kind == "op" and \
                        self.toks[self._next_index()].value in ("=", ":"):
                    self.next()
                    key = Literal(ktok.value)
                else:
                    key = self.parse_expr()
                sep = self.next()
                if sep.kind != "op" or sep.value not in ("=", ":"):
                    self.error("expected '=' in object", sep)
                value = self.parse_expr()
                items.append((key, value))
                if self.peek().kind == "op" and self.peek().value == ",":
                    self.next()
            self.expect_op("}")
            self.nl_depth -= 1
            return ObjectExpr(items)
        self.error("unexpected token %r" % (tok.value,), tok)

    def _next_index(self) -> int:
        """Index of the token after the next non-newline token."""
        j = self.i
        while self.toks[j].kind == "nl":
            j += 1
        j += 1
        while self.toks[j].kind == "nl":
            j += 1
        return j

    def parse_for(self, is_object: bool):
        self.next()  # 'for'
        first = self.next()
        key_var, value_var = None, first.value
        if self.peek().kind == "op" and self.peek().value == ",":
            self.next()
            key_var, value_var = first.value, self.next().value
        tok = self.next()
        if tok.kind != "ident" or tok.value != "in":
            self.error("expected 'in'", tok)
        collection = self.parse_expr()
        self.expect_op(":")
        key_expr = None
        if is_object:
            key_expr = self.parse_expr()
            self.expect_op("=>")
        value_expr = self.parse_expr()
        if self.peek().kind == "op" and self.peek().value == "...":
            self.next()
        cond = None
        if self.peek().kind == "ident" and self.peek().value == "if":
            self.next()
            cond = self.parse_expr()
        self.expect_op("}" if is_object else "]")
        return ForExpr(key_var, value_var, collection, key_expr, value_expr, cond, is_object)


def parse(src: str, filename: str = "") -> Body:
    return Parser(tokenize(src, filename), filename).parse_body(None)


def parse_expression(src: str, filename: str = "", line: int = 0):
    parser = Parser(tokenize(src, filename), filename)
    parser.nl_depth = 1
    expr = parser.parse_expr()
    if parser.peek().kind != "eof":
        raise HCLSyntaxError("unexpected trailing input in expression %r" % src, line, filename)
    return expr


def parse_file(path: str) -> Body:
    with open(path) as handle:
        return parse(handle.read(), path)
