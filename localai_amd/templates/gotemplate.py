"""A Go `text/template` interpreter (plus the sprig functions LocalAI templates use).

LocalAI renders prompts with Go templates + sprig (`pkg/templates/cache.go:97`); every
gallery / embedded model YAML depends on their exact semantics:
`{{-`/`-}}` whitespace trimming, if / else if / range / with, `$x :=` variables,
variadic `eq`, Go truthiness, sorted map ranges, `print`'s Sprint spacing, and sprig
`toJson` (compact, HTML-escaped, sorted keys).  Data are Python dicts / objects whose
keys / attributes use the Go field names (`.RoleName`, `.Content`, ...).
"""
from __future__ import annotations

import json
import math
import re
from typing import Any, Callable, Dict, List, Optional, Tuple


class TemplateError(Exception):
    pass


class _NoValue:
    def __repr__(self):
        return "<no value>"

    def __bool__(self):
        return False


NO_VALUE = _NoValue()


# ------------------------------------------------------------------------------ lexing
_ACTION_RE = re.compile(r"\{\{(-\s)?(.*?)(\s-)?\}\}", re.S)


def _split(src: str) -> List[Tuple[str, str]]:
    """-> [("text", s) | ("action", body)], applying {{- / -}} trimming."""
    out: List[Tuple[str, str]] = []
    pos = 0
    trim_next = False
    i = 0
    n = len(src)
    while True:
        j = src.find("{{", pos)
        if j < 0:
            text = src[pos:]
            if trim_next:
                text = text.lstrip(" \t\r\n")
            if text:
                out.append(("text", text))
            break
        # find matching close, skipping over string literals and comments
        k = j + 2
        trim_left = False
        if k < n and src[k] == "-" and k + 1 < n and src[k + 1] in " \t\r\n":
            trim_left = True
            k += 2
        body_start = k
        end = None
        in_str = None
        while k < n:
            c = src[k]
            if in_str:
                if c == "\\" and in_str == '"':
                    k += 2
                    continue
                if c == in_str:
                    in_str = None
                k += 1
                continue
            if c in "\"`'":
                in_str = c
                k += 1
                continue
            if src.startswith("/*", k):
                e = src.find("*/", k + 2)
                if e < 0:
                    raise TemplateError("unclosed comment")
                k = e + 2
                continue
            if src.startswith("}}", k):
                end = k
                break
            k += 1
        if end is None:
            raise TemplateError("unclosed action")
        body = src[body_start:end]
        trim_right = False
        if len(body) >= 2 and body[-1] == "-" and body[-2] in " \t\r\n":
            trim_right = True
            body = body[:-2]
        text = src[pos:j]
        if trim_next:
            text = text.lstrip(" \t\r\n")
        if trim_left:
            text = text.rstrip(" \t\r\n")
        if text:
            out.append(("text", text))
        out.append(("action", body))
        trim_next = trim_right
        pos = end + 2
    return out


_TOK_RE = re.compile(r"""
    (?P<ws>\s+)
  | (?P<comment>/\*.*?\*/)
  | (?P<raw>`[^`]*`)
  | (?P<str>"(?:\\.|[^"\\])*")
  | (?P<char>'(?:\\.|[^'\\])')
  | (?P<declare>:=)
  | (?P<assign>=)
  | (?P<num>[+-]?(?:0[xX][0-9a-fA-F]+|\d+\.?\d*(?:[eE][+-]?\d+)?|\.\d+(?:[eE][+-]?\d+)?))
  | (?P<var>\$[A-Za-z0-9_]*)
  | (?P<field>(?:\.[A-Za-z_][A-Za-z0-9_]*)+)
  | (?P<dot>\.)
  | (?P<ident>[A-Za-z_][A-Za-z0-9_]*)
  | (?P<lp>\()
  | (?P<rp>\))
  | (?P<pipe>\|)
  | (?P<comma>,)
""", re.X | re.S)


def _tokenize(s: str):
    toks = []
    pos = 0
    glued = False
    while pos < len(s):
        m = _TOK_RE.match(s, pos)
        if not m:
            raise TemplateError(f"bad token at {s[pos:pos + 20]!r}")
        kind = m.lastgroup
        val = m.group(kind)
        pos = m.end()
        if kind in ("ws", "comment"):
            glued = False
            continue
        # a field chain written directly after a variable or ")" (no space) is a selector
        if kind == "field" and glued and toks and toks[-1][0] in ("var", "rp"):
            kind = "selector"
        toks.append((kind, val))
        glued = True
    return toks


# ------------------------------------------------------------------------------ AST
class Node:
    pass


class Text(Node):
    def __init__(self, s):
        self.s = s


class Action(Node):
    def __init__(self, pipe):
        self.pipe = pipe


class If(Node):
    def __init__(self, pipe, body, els, kind="if"):
        self.pipe, self.body, self.els, self.kind = pipe, body, els, kind


class Range(Node):
    def __init__(self, pipe, body, els):
        self.pipe, self.body, self.els = pipe, body, els


class Pipeline:
    def __init__(self, decl, is_assign, cmds):
        self.decl, self.is_assign, self.cmds = decl, is_assign, cmds


class Cmd:
    def __init__(self, args):
        self.args = args


# operand kinds
class Lit:
    def __init__(self, v):
        self.v = v


class FieldRef:  # .A.B  (on dot)
    def __init__(self, names):
        self.names = names


class VarRef:  # $x.A.B
    def __init__(self, name, names):
        self.name, self.names = name, names


class Ident:
    def __init__(self, name):
        self.name = name


class SubPipe:
    def __init__(self, pipe, names):
        self.pipe, self.names = pipe, names


class Dot:
    pass


def _unquote(s: str) -> str:
    if s[0] == "`":
        return s[1:-1]
    return json.loads(s) if s[0] == '"' else s


class _Parser:
    def __init__(self, pieces):
        self.pieces = pieces
        self.i = 0

    def parse_list(self, stop=("end", "else")) -> Tuple[List[Node], Optional[str], Optional[list]]:
        nodes: List[Node] = []
        while self.i < len(self.pieces):
            kind, val = self.pieces[self.i]
            self.i += 1
            if kind == "text":
                nodes.append(Text(val))
                continue
            toks = _tokenize(val)
            if not toks:
                continue  # comment-only action
            head = toks[0]
            if head == ("ident", "end"):
                return nodes, "end", None
            if head == ("ident", "else"):
                return nodes, "else", toks[1:]
            if head == ("ident", "if") or head == ("ident", "with"):
                nodes.append(self._parse_if(toks[1:], head[1]))
                continue
            if head == ("ident", "range"):
                pipe = self._pipeline(toks[1:])
                body, term, rest = self.parse_list()
                els = []
                if term == "else":
                    els, term, _ = self.parse_list()
                nodes.append(Range(pipe, body, els))
                continue
            if head[0] == "ident" and head[1] in ("define", "template", "block"):
                raise TemplateError(f"{head[1]} is not supported")
            if head[0] == "ident" and head[1] in ("break", "continue"):
                nodes.append(Action(Pipeline([], False, [Cmd([Ident("__" + head[1])])])))
                continue
            nodes.append(Action(self._pipeline(toks)))
        return nodes, None, None

    def _parse_if(self, toks, kind):
        pipe = self._pipeline(toks)
        body, term, rest = self.parse_list()
        els: List[Node] = []
        if term == "else":
            if rest and rest[0] in (("ident", "if"), ("ident", "with")):
                # else if / else with: the chain shares the single {{end}}
                els = [self._parse_if(rest[1:], rest[0][1])]
            else:
                els, term, _ = self.parse_list()
        return If(pipe, body, els, kind)

    def _pipeline(self, toks) -> Pipeline:
        decl: List[str] = []
        is_assign = False
        # declarations: $a := / $a, $b := / $a =
        j = 0
        vars_ = []
        while j < len(toks) and toks[j][0] == "var":
            vars_.append(toks[j][1])
            if j + 1 < len(toks) and toks[j + 1][0] == "comma":
                j += 2
                continue
            j += 1
            break
        if vars_ and j < len(toks) and toks[j][0] in ("declare", "assign"):
            decl = vars_
            is_assign = toks[j][0] == "assign"
            toks = toks[j + 1:]
        cmds = []
        cur: List = []
        k = 0
        while k < len(toks):
            kind, val = toks[k]
            if kind == "pipe":
                cmds.append(Cmd(cur))
                cur = []
                k += 1
                continue
            op, k = self._operand(toks, k)
            cur.append(op)
        if cur:
            cmds.append(Cmd(cur))
        return Pipeline(decl, is_assign, cmds)

    def _operand(self, toks, k):
        kind, val = toks[k]
        k += 1
        if kind == "lp":
            depth = 1
            j = k
            while j < len(toks) and depth:
                if toks[j][0] == "lp":
                    depth += 1
                elif toks[j][0] == "rp":
                    depth -= 1
                j += 1
            inner = self._pipeline(toks[k:j - 1])
            names = []
            if j < len(toks) and toks[j][0] == "selector":
                names = toks[j][1].split(".")[1:]
                j += 1
            return SubPipe(inner, names), j
        if kind == "field":
            return FieldRef(val.split(".")[1:]), k
        if kind == "dot":
            return Dot(), k
        if kind == "var":
            names = []
            if k < len(toks) and toks[k][0] == "selector":
                names = toks[k][1].split(".")[1:]
                k += 1
            return VarRef(val, names), k
        if kind in ("str", "raw"):
            return Lit(_unquote(val)), k
        if kind == "char":
            return Lit(ord(json.loads('"' + val[1:-1] + '"'))), k
        if kind == "num":
            if re.fullmatch(r"[+-]?\d+", val) or val.lower().startswith(("0x", "+0x", "-0x")):
                return Lit(int(val, 0)), k
            return Lit(float(val)), k
        if kind == "ident":
            if val == "true":
                return Lit(True), k
            if val == "false":
                return Lit(False), k
            if val == "nil":
                return Lit(None), k
            return Ident(val), k
        raise TemplateError(f"unexpected token {val!r}")


# ------------------------------------------------------------------------------ values
def truth(v) -> bool:
    if v is None or v is NO_VALUE:
        return False
    if isinstance(v, bool):
        return v
    if isinstance(v, (int, float)):
        return v != 0
    if isinstance(v, (str, list, tuple, dict, bytes)):
        return len(v) > 0
    return True


def _fmt_float(f: float) -> str:
    if math.isinf(f):
        return "+Inf" if f > 0 else "-Inf"
    if math.isnan(f):
        return "NaN"
    if f == int(f) and abs(f) < 1e21:
        return str(int(f))
    r = repr(f)
    if "e" in r:
        mant, exp = r.split("e")
        sign = "-" if exp.startswith("-") else "+"
        exp = exp.lstrip("+-").lstrip("0").rjust(2, "0")
        return f"{mant}e{sign}{exp}"
    return r


def go_str(v) -> str:
    """fmt %v formatting."""
    if v is NO_VALUE:
        return "<no value>"
    if v is None:
        return "<nil>"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float):
        return _fmt_float(v)
    if isinstance(v, (list, tuple)):
        return "[" + " ".join(go_str(x) for x in v) + "]"
    if isinstance(v, dict):
        return "map[" + " ".join(f"{go_str(k)}:{go_str(v[k])}" for k in sorted(v, key=str)) + "]"
    return str(v)


def _json_default(o):
    if hasattr(o, "to_json"):
        return o.to_json()
    if hasattr(o, "__dict__"):
        return {k: v for k, v in o.__dict__.items() if not k.startswith("_")}
    raise TypeError(str(type(o)))


def _go_json(v) -> str:
    """encoding/json.Marshal: compact, sorted map keys, HTML-safe escaping, integral floats."""
    def conv(x):
        if isinstance(x, float) and x == int(x) and abs(x) < 1e21:
            return int(x)
        if isinstance(x, dict):
            return {str(k): conv(val) for k, val in x.items()}
        if isinstance(x, (list, tuple)):
            return [conv(val) for val in x]
        if x is NO_VALUE:
            return None
        if not isinstance(x, (str, int, float, bool)) and x is not None:
            return conv(_json_default(x))
        return x
    s = json.dumps(conv(v), separators=(",", ":"), sort_keys=True, ensure_ascii=False)
    return (s.replace("<", "\\u003c").replace(">", "\\u003e").replace("&", "\\u0026")
            .replace("\u2028", "\\u2028").replace("\u2029", "\\u2029"))


def _sprint(args) -> str:
    # fmt.Sprint: spaces between operands when neither side is a string
    out = []
    prev_str = True
    for i, a in enumerate(args):
        is_str = isinstance(a, str)
        if i > 0 and not is_str and not prev_str:
            out.append(" ")
        out.append(go_str(a))
        prev_str = is_str
    return "".join(out)


def _printf(fmt: str, *args) -> str:
    args = list(args)
    out = []
    i = 0
    ai = 0
    while i < len(fmt):
        c = fmt[i]
        if c != "%":
            out.append(c)
            i += 1
            continue
        i += 1
        if i < len(fmt) and fmt[i] == "%":
            out.append("%")
            i += 1
            continue
        m = re.match(r"([-+ #0]*)(\d*)(?:\.(\d+))?([a-zA-Z])", fmt[i:])
        if not m:
            out.append("%")
            continue
        flags, width, prec, verb = m.groups()
        i += m.end()
        a = args[ai] if ai < len(args) else NO_VALUE
        ai += 1
        if verb in ("v", "s"):
            s = go_str(a)
        elif verb == "d":
            s = str(int(a))
        elif verb in ("f", "F"):
            s = f"{float(a):.{int(prec) if prec else 6}f}"
        elif verb == "q":
            s = json.dumps(str(a), ensure_ascii=False)
        elif verb == "t":
            s = go_str(bool(a))
        elif verb == "x":
            s = a.encode().hex() if isinstance(a, str) else format(int(a), "x")
        else:
            s = go_str(a)
        if width:
            s = s.ljust(int(width)) if "-" in flags else s.rjust(int(width))
        out.append(s)
    return "".join(out)


def _eq(a, *bs):
    for b in bs:
        if a == b and type(a) is type(b) or (isinstance(a, (int, float)) and isinstance(b, (int, float))
                                              and not isinstance(a, bool) and a == b):
            return True
        if a == b and not isinstance(a, (int, float)):
            return True
    return False


def _index(c, *keys):
    for k in keys:
        if isinstance(c, dict):
            c = c.get(k, NO_VALUE)
        elif isinstance(c, (list, tuple, str)):
            c = c[int(k)]
        else:
            c = getattr(c, str(k), NO_VALUE)
    return c


def _default(d, v=NO_VALUE):
    return v if truth(v) else d


FUNCS: Dict[str, Callable] = {
    "eq": _eq,
    "ne": lambda a, b: not _eq(a, b),
    "lt": lambda a, b: a < b,
    "le": lambda a, b: a <= b,
    "gt": lambda a, b: a > b,
    "ge": lambda a, b: a >= b,
    "not": lambda a: not truth(a),
    "len": lambda a: len(a),
    "index": _index,
    "print": lambda *a: _sprint(a),
    "println": lambda *a: " ".join(go_str(x) for x in a) + "\n",
    "printf": _printf,
    "html": lambda *a: _sprint(a).replace("&", "&amp;").replace("<", "&lt;").replace(">", "&gt;")
    .replace('"', "&#34;").replace("'", "&#39;"),
    "urlquery": lambda *a: __import__("urllib.parse").parse.quote_plus(_sprint(a)),
    "js": lambda *a: json.dumps(_sprint(a))[1:-1],
    "slice": lambda c, *ix: c[ix[0]:ix[1]] if len(ix) == 2 else c[ix[0]:] if ix else c,
    # sprig subset
    "toJson": _go_json,
    "toPrettyJson": lambda v: json.dumps(v, indent=2, sort_keys=True, ensure_ascii=False),
    "toString": go_str,
    "trim": lambda s: go_str(s).strip(),
    "trimAll": lambda c, s: go_str(s).strip(c),
    "trimSuffix": lambda suf, s: s[:-len(suf)] if suf and s.endswith(suf) else s,
    "trimPrefix": lambda pre, s: s[len(pre):] if pre and s.startswith(pre) else s,
    "upper": lambda s: go_str(s).upper(),
    "lower": lambda s: go_str(s).lower(),
    "title": lambda s: go_str(s).title(),
    "replace": lambda old, new, s: go_str(s).replace(old, new),
    "contains": lambda sub, s: sub in go_str(s),
    "hasPrefix": lambda p, s: go_str(s).startswith(p),
    "hasSuffix": lambda p, s: go_str(s).endswith(p),
    "quote": lambda *a: " ".join(json.dumps(go_str(x), ensure_ascii=False) for x in a),
    "squote": lambda *a: " ".join("'" + go_str(x) + "'" for x in a),
    "default": _default,
    "empty": lambda v: not truth(v),
    "join": lambda sep, l: sep.join(go_str(x) for x in l),
    "split": lambda sep, s: {f"_{i}": p for i, p in enumerate(go_str(s).split(sep))},
    "splitList": lambda sep, s: go_str(s).split(sep),
    "list": lambda *a: list(a),
    "dict": lambda *a: {a[i]: a[i + 1] for i in range(0, len(a) - 1, 2)},
    "add": lambda *a: sum(a),
    "add1": lambda a: a + 1,
    "sub": lambda a, b: a - b,
    "mul": lambda *a: math.prod(a),
    "div": lambda a, b: a // b,
    "mod": lambda a, b: a % b,
    "max": lambda *a: max(a),
    "min": lambda *a: min(a),
    "repeat": lambda n, s: s * n,
    "nospace": lambda s: re.sub(r"\s", "", s),
    "indent": lambda n, s: "\n".join(" " * n + l for l in s.split("\n")),
    "nindent": lambda n, s: "\n" + "\n".join(" " * n + l for l in s.split("\n")),
    "ternary": lambda a, b, c: a if truth(c) else b,
    "coalesce": lambda *a: next((x for x in a if truth(x)), None),
    "first": lambda l: l[0] if l else None,
    "last": lambda l: l[-1] if l else None,
    "keys": lambda d: sorted(d.keys()),
    "hasKey": lambda d, k: k in d,
    "toStrings": lambda l: [go_str(x) for x in l],
    "regexMatch": lambda r, s: re.search(r, s) is not None,
    "regexReplaceAll": lambda r, s, rep: re.sub(r, rep.replace("$", "\\"), s),
    "b64enc": lambda s: __import__("base64").b64encode(go_str(s).encode()).decode(),
    "b64dec": lambda s: __import__("base64").b64decode(s).decode(),
    "fromJson": lambda s: json.loads(s),
}


class _Break(Exception):
    pass


class _Continue(Exception):
    pass


class Template:
    def __init__(self, src: str, funcs: Optional[Dict[str, Callable]] = None):
        self.src = src
        self.funcs = dict(FUNCS)
        if funcs:
            self.funcs.update(funcs)
        p = _Parser(_split(src))
        nodes, term, _ = p.parse_list()
        if term is not None:
            raise TemplateError(f"unexpected {{{{{term}}}}}")
        self.nodes = nodes

    def execute(self, data: Any) -> str:
        out: List[str] = []
        scope = [{"$": data}]
        self._run(self.nodes, data, scope, out)
        return "".join(out)

    # -------------------------------------------------------------- evaluation
    def _lookup_var(self, scope, name):
        for s in reversed(scope):
            if name in s:
                return s[name]
        raise TemplateError(f"undefined variable {name}")

    def _set_var(self, scope, name, v):
        for s in reversed(scope):
            if name in s:
                s[name] = v
                return
        raise TemplateError(f"undefined variable {name}")

    @staticmethod
    def _field(v, name):
        if v is None or v is NO_VALUE:
            return NO_VALUE
        if isinstance(v, dict):
            return v.get(name, NO_VALUE)
        if hasattr(v, name):
            return getattr(v, name)
        raise TemplateError(f"can't evaluate field {name} in type {type(v).__name__}")

    def _chain(self, v, names):
        for n in names:
            v = self._field(v, n)
        return v

    def _operand(self, op, dot, scope):
        if isinstance(op, Lit):
            return op.v
        if isinstance(op, Dot):
            return dot
        if isinstance(op, FieldRef):
            return self._chain(dot, op.names)
        if isinstance(op, VarRef):
            return self._chain(self._lookup_var(scope, op.name), op.names)
        if isinstance(op, SubPipe):
            return self._chain(self._pipe(op.pipe, dot, scope), op.names)
        if isinstance(op, Ident):
            return self._call(op.name, [], dot, scope)
        raise TemplateError("bad operand")

    def _call(self, name, args, dot, scope):
        if name == "__break":
            raise _Break()
        if name == "__continue":
            raise _Continue()
        if name in ("and", "or"):
            # short-circuit semantics of Go 1.18+: returns first falsy/truthy arg
            last = None
            for a in args:
                last = self._operand(a, dot, scope) if not isinstance(a, _Evald) else a.v
                if name == "and" and not truth(last):
                    return last
                if name == "or" and truth(last):
                    return last
            return last
        fn = self.funcs.get(name)
        if fn is None:
            raise TemplateError(f'function "{name}" not defined')
        vals = [a.v if isinstance(a, _Evald) else self._operand(a, dot, scope) for a in args]
        return fn(*vals)

    def _pipe(self, pipe: Pipeline, dot, scope):
        val = None
        have = False
        for cmd in pipe.cmds:
            args = list(cmd.args)
            if have:
                args = args + [_Evald(val)]
            first = args[0]
            if isinstance(first, Ident):
                val = self._call(first.name, args[1:], dot, scope)
            else:
                if len(args) > 1:
                    raise TemplateError("can't give argument to non-function")
                val = first.v if isinstance(first, _Evald) else self._operand(first, dot, scope)
            have = True
        if pipe.decl:
            if pipe.is_assign:
                self._set_var(scope, pipe.decl[0], val)
            else:
                scope[-1][pipe.decl[-1]] = val
        return val

    def _run(self, nodes, dot, scope, out):
        for n in nodes:
            if isinstance(n, Text):
                out.append(n.s)
            elif isinstance(n, Action):
                v = self._pipe(n.pipe, dot, scope)
                if not n.pipe.decl:
                    out.append(go_str(v))
            elif isinstance(n, If):
                scope.append({})
                try:
                    v = self._pipe(n.pipe, dot, scope)
                    if truth(v):
                        self._run(n.body, v if n.kind == "with" else dot, scope, out)
                    else:
                        self._run(n.els, dot, scope, out)
                finally:
                    scope.pop()
            elif isinstance(n, Range):
                scope.append({})
                try:
                    decl = n.pipe.decl
                    p2 = Pipeline([], False, n.pipe.cmds)
                    v = self._pipe(p2, dot, scope)
                    if isinstance(v, dict):
                        items = [(k, v[k]) for k in sorted(v, key=lambda x: (str(type(x)), x))]
                    elif isinstance(v, int) and not isinstance(v, bool):
                        items = list(enumerate(range(v)))
                    elif v is None or v is NO_VALUE:
                        items = []
                    else:
                        items = list(enumerate(v))
                    if not items:
                        self._run(n.els, dot, scope, out)
                    for k, e in items:
                        if len(decl) == 1:
                            scope[-1][decl[0]] = e
                        elif len(decl) >= 2:
                            scope[-1][decl[0]] = k
                            scope[-1][decl[1]] = e
                        try:
                            self._run(n.body, e, scope, out)
                        except _Continue:
                            continue
                        except _Break:
                            break
                finally:
                    scope.pop()


class _Evald:
    def __init__(self, v):
        self.v = v


def render(src: str, data: Any) -> str:
    return Template(src).execute(data)
