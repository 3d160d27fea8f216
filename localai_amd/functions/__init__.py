"""OpenAI functions/tools -> JSON-schema `oneOf` -> GBNF grammar, and function-call parsing of
model output (`pkg/functions/*`: functions.go, function_structure.go, parse.go,
grammars/{json_schema,llama31_schema,rules,bnf_rules,options}.go).

The grammar text is produced rule-for-rule like the reference (same rule names such as
`root-0-arguments`, `space ::= " "?`, `freestring`, `mixedstring`, `arr`) so grammars written
for LocalAI keep working; it is consumed by our GBNF engine (localai_amd/grammar).
Rules are emitted in a deterministic order (Go ranges a map, so its order is random).
"""
from __future__ import annotations

import json
import re
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

DEFAULT_NAME_KEY = "name"
DEFAULT_ARGS_KEY = "arguments"

JSON_BNF = r'''root   ::= object
value  ::= object | array | string | number | ("true" | "false" | "null") ws

object ::=
  "{" ws (
            string ":" ws value
    ("," ws string ":" ws value)*
  )? "}" ws

array  ::=
  "[" ws (
            value
    ("," ws value)*
  )? "]" ws

string ::=
  "\"" (
    [^"\\] |
    "\\" (["\\/bfnrt] | "u" [0-9a-fA-F] [0-9a-fA-F] [0-9a-fA-F] [0-9a-fA-F]) # escapes
  )* "\"" ws

number ::= ("-"? ([0-9] | [1-9] [0-9]*)) ("." [0-9]+)? ([eE] [-+]? [0-9]+)? ws

ws ::= ([ \t\n] ws)?'''

PRIMITIVE_RULES = {
    "boolean": '("true" | "false") space',
    "number": '("-"? ([0-9] | [1-9] [0-9]*)) ("." [0-9]+)? ([eE] [-+]? [0-9]+)? space',
    "integer": '("-"? ([0-9] | [1-9] [0-9]*)) space',
    "string": '"\\"" (\n\t\t\t[^"\\\\] |\n\t\t\t"\\\\" (["\\\\/bfnrt] | "u" [0-9a-fA-F] [0-9a-fA-F] [0-9a-fA-F] '
              '[0-9a-fA-F])\n\t\t  )* "\\"" space',
    "freestring": '(\n\t\t\t[^\\x00] |\n\t\t\t"\\\\" (["\\\\/bfnrt] | "u" [0-9a-fA-F] [0-9a-fA-F] [0-9a-fA-F] '
                  '[0-9a-fA-F])\n\t\t  )* space',
    "null": '"null" space',
}
SPACE_RULE = '" "?'
ARRAY_NEWLINES = 'arr  ::=\n  "[\\n"  (\n\t\trealvalue\n    (",\\n"  realvalue)*\n  )? "]"'
ARRAY = 'arr  ::=\n  "["  (\n\t\trealvalue\n    (","  realvalue)*\n  )? "]"'

INVALID_RULE_CHARS_RE = re.compile(r"[^a-zA-Z0-9-]+")
GRAMMAR_LITERAL_ESCAPE_RE = re.compile(r'[\r\n"]')
GRAMMAR_LITERAL_ESCAPES = {"\r": "\\r", "\n": "\\n", '"': '\\"'}
LLAMA31 = "llama3.1"

_DQ_RE = re.compile(r'"[^"\\]*(?:\\[\s\S][^"\\]*)*"')
_NL_RE = re.compile(r"[\r\n]")


def escape_new_lines(s: str) -> str:
    """utils.EscapeNewLines: escape raw newlines inside double-quoted strings."""
    return _DQ_RE.sub(lambda m: _NL_RE.sub("\\\\n", m.group(0)), s)


def _go_json(v) -> str:
    from ..templates.gotemplate import _go_json as gj
    return gj(v)


@dataclass
class GrammarOptions:
    prop_order: str = ""
    prefix: str = ""
    maybe_array: bool = False
    disable_parallel_new_lines: bool = False
    maybe_string: bool = False
    no_mixed_free_string: bool = False
    expect_strings_after_json: bool = False
    function_name: str = ""
    schema_type: str = "json"


class Rules(dict):
    def to_grammar(self, o: GrammarOptions) -> str:
        prefix = o.prefix
        swap_root = o.maybe_array or o.maybe_string or prefix != ""
        lines = []
        for name, rule in self.items():
            if swap_root and name == "root":
                name = "realvalue"
            lines.append(f"{name} ::= {rule}")
        if not swap_root:
            return "\n".join(lines)
        new_root = "realvalue"
        if o.maybe_array:
            new_root = "arr | realvalue"
        free = "freestring" if o.no_mixed_free_string else "mixedstring"
        if prefix:
            prefix = escape_new_lines(prefix)
            if o.maybe_array and o.maybe_string:
                new_root = "(" + new_root + ")"
            if o.maybe_string:
                new_root = '( "' + prefix + '" ' + new_root + " | " + free + " ) "
            else:
                new_root = '"' + prefix + '" ' + new_root
        elif o.maybe_string:
            new_root = free + " | " + new_root
        lines.append(f"root ::= {new_root}")
        lines.append(ARRAY if o.disable_parallel_new_lines else ARRAY_NEWLINES)
        if o.maybe_array:
            if o.expect_strings_after_json:
                lines.append("mixedstring ::= freestring | freestring arr freestring | "
                             "(freestring realvalue freestring)* | realvalue | arr")
            else:
                lines.append("mixedstring ::= freestring | freestring arr | freestring realvalue | realvalue | arr")
        else:
            if o.expect_strings_after_json:
                lines.append("mixedstring ::= freestring | (freestring realvalue freestring)* | realvalue")
            else:
                lines.append("mixedstring ::= freestring | freestring realvalue | realvalue")
        return "\n".join(lines)


class _ConverterBase:
    def __init__(self):
        self.rules = Rules()
        self.rules["space"] = SPACE_RULE

    def add_rule(self, name: str, rule: str) -> str:
        esc = INVALID_RULE_CHARS_RE.sub("-", name)
        key = esc
        if esc in self.rules and self.rules[esc] != rule:
            i = 0
            while f"{esc}{i}" in self.rules:
                i += 1
            key = f"{esc}{i}"
        self.rules[key] = rule
        return key

    @staticmethod
    def resolve_ref(ref: str, root: dict) -> dict:
        if not ref.startswith("#/$defs/"):
            raise ValueError(f"invalid reference format: {ref}")
        defs = root.get("$defs")
        if not isinstance(defs, dict):
            raise ValueError("no definitions found in the schema")
        d = defs.get(ref[len("#/$defs/"):])
        if not isinstance(d, dict):
            raise ValueError(f"definition not found: {ref}")
        return d

    @staticmethod
    def format_literal_quoted(v) -> str:
        j = _go_json(v)
        return '"' + GRAMMAR_LITERAL_ESCAPE_RE.sub(lambda m: GRAMMAR_LITERAL_ESCAPES[m.group(0)], j) + '"'

    def grammar(self, schema: dict, o: GrammarOptions) -> str:
        self.add_rule("freestring", PRIMITIVE_RULES["freestring"])
        self.visit(schema, "", schema)
        return self.rules.to_grammar(o)

    def _alternatives(self, schema, rule_name, root):
        alts = []
        lst = schema.get("oneOf") if isinstance(schema.get("oneOf"), list) else schema.get("anyOf")
        for i, alt in enumerate(lst or []):
            alts.append(self.visit(alt, f"{rule_name}-{i}", root))
        return self.add_rule(rule_name, " | ".join(alts))

    def _primitive(self, schema, rule_name):
        st = schema.get("type", "")
        if st not in PRIMITIVE_RULES:
            raise ValueError(f"unrecognized schema: {schema}")
        if rule_name == "root":
            st = "root"
        return self.add_rule(st, PRIMITIVE_RULES[schema.get("type")])


class JSONSchemaConverter(_ConverterBase):
    def __init__(self, prop_order: str = ""):
        super().__init__()
        self.prop_order = {n: i for i, n in enumerate(prop_order.split(","))}

    def visit(self, schema: dict, name: str, root: dict) -> str:
        st = schema.get("type", "")
        rule_name = name or "root"
        if "oneOf" in schema or "anyOf" in schema:
            return self._alternatives(schema, rule_name, root)
        if isinstance(schema.get("$ref"), str):
            return self.visit(self.resolve_ref(schema["$ref"], root), name, root)
        if "const" in schema:
            return self.add_rule(rule_name, self.format_literal_quoted(schema["const"]))
        if isinstance(schema.get("enum"), list):
            return self.add_rule(rule_name, " | ".join(self.format_literal_quoted(v) for v in schema["enum"]))
        if st == "object" and isinstance(schema.get("properties"), dict):
            po = self.prop_order
            pairs = list(schema["properties"].items())

            def key(p):
                return p[0]
            # Go: sort.Slice with "both have an order => by order, else by name"
            import functools

            def cmp(a, b):
                ia, ib = po.get(a[0], 0), po.get(b[0], 0)
                if ia != 0 and ib != 0:
                    return -1 if ia < ib else (1 if ia > ib else 0)
                return -1 if a[0] < b[0] else (1 if a[0] > b[0] else 0)
            pairs.sort(key=functools.cmp_to_key(cmp))
            parts = ['"{" space']
            for i, (pn, ps) in enumerate(pairs):
                prn = self.visit(ps, f"{rule_name}-{pn}", root)
                if i > 0:
                    parts.append(' "," space')
                parts.append(f' {self.format_literal_quoted(pn)} space ":" space {prn}')
            parts.append(' "}" space')
            return self.add_rule(rule_name, "".join(parts))
        if st == "array" and isinstance(schema.get("items"), dict):
            item = self.visit(schema["items"], f"{rule_name}-item", root)
            return self.add_rule(rule_name, f'"[" space ({item} ("," space {item})*)? "]" space')
        return self._primitive(schema, rule_name)


class LLama31SchemaConverter(_ConverterBase):
    """Emits llama3.1-style `<function=name>{...}</function>` calls."""

    def __init__(self, fn_name: str = ""):
        super().__init__()
        self.fn_name = fn_name or "name"

    @staticmethod
    def format_literal(v) -> str:
        return re.sub(r"[\r\n]", lambda m: {"\r": "\\r", "\n": "\\n"}[m.group(0)], _go_json(v))

    def visit(self, schema: dict, name: str, root: dict) -> str:
        st = schema.get("type", "")
        rule_name = name or "root"
        if "oneOf" in schema or "anyOf" in schema:
            return self._alternatives(schema, rule_name, root)
        if isinstance(schema.get("$ref"), str):
            return self.visit(self.resolve_ref(schema["$ref"], root), name, root)
        if "const" in schema:
            return self.add_rule(rule_name, self.format_literal(schema["const"]))
        if isinstance(schema.get("enum"), list):
            return self.add_rule(rule_name, " | ".join(self.format_literal_quoted(v) for v in schema["enum"]))
        if st == "object" and isinstance(schema.get("properties"), dict):
            base = len(name.split("-")) == 2
            pairs = sorted(schema["properties"].items(), key=lambda p: p[0])
            parts = ['"<function="' if base else '"{" space']
            if base:
                name_pair = None
                for i, p in enumerate(pairs):
                    if p[0] == self.fn_name:
                        name_pair = p
                        pairs.pop(i)
                        break
                if name_pair is None:
                    raise ValueError(f"no function name found in the schema: {schema}")
                prn = self.visit(name_pair[1], f"{rule_name}-{self.fn_name}", root)
                parts.append(f' {prn} ">{{" ')
                for pn, ps in pairs:
                    parts.append(self.visit(ps, f"{rule_name}-{pn}", root))
                parts.append(' "}</function>"')
            else:
                for i, (pn, ps) in enumerate(pairs):
                    prn = self.visit(ps, f"{rule_name}-{pn}", root)
                    if i > 0:
                        parts.append(' "," space')
                    parts.append(f' {self.format_literal_quoted(pn)} space ":" space {prn}')
                parts.append(' "}" space')
            return self.add_rule(rule_name, "".join(parts))
        if st == "array" and isinstance(schema.get("items"), dict):
            item = self.visit(schema["items"], f"{rule_name}-item", root)
            return self.add_rule(rule_name, f'"[" space ({item} ("," space {item})*)? "]" space')
        return self._primitive(schema, rule_name)


# --------------------------------------------------------------------------- structures
def _json_roundtrip(v):
    return json.loads(json.dumps(v)) if v is not None else None


def to_json_structure(functions: List[dict], name_key: str = "", args_key: str = "") -> dict:
    """Functions.ToJSONStructure: oneOf over {name: {const}, arguments: {type: object, properties}}."""
    nk = name_key or DEFAULT_NAME_KEY
    ak = args_key or DEFAULT_ARGS_KEY
    js: Dict[str, Any] = {"oneOf": []}
    defs_set = False
    for f in functions:
        params = f.get("parameters") or {}
        prop = _json_roundtrip(params.get("properties")) or {}
        defs = _json_roundtrip(params.get("$defs")) or {}
        if not defs_set:
            js["$defs"] = defs
            defs_set = True
        js["oneOf"].append({"type": "object", "properties": {
            nk: {"const": f.get("name", "")},
            ak: {"type": "object", "properties": prop}}})
    if not js.get("$defs"):
        js.pop("$defs", None)
    if not js["oneOf"]:
        js.pop("oneOf")
    return js


def select(functions: List[dict], name: str) -> List[dict]:
    for f in functions:
        if f.get("name") == name:
            return [f]
    return []


def grammar_options(fcfg: Optional[dict]) -> GrammarOptions:
    fcfg = fcfg or {}
    g = fcfg.get("grammar") or {}
    return GrammarOptions(
        prop_order=str(g.get("properties_order") or ""),
        prefix=str(g.get("prefix") or ""),
        maybe_array=bool(g.get("parallel_calls")),
        disable_parallel_new_lines=bool(g.get("disable_parallel_new_lines")),
        maybe_string=bool(g.get("mixed_mode")),
        no_mixed_free_string=bool(g.get("no_mixed_free_string")),
        expect_strings_after_json=bool(g.get("expect_strings_after_json")),
        function_name=str(fcfg.get("function_name_key") or ""),
        schema_type=str(g.get("schema_type") or "json"),
    )


def structure_grammar(structure: dict, opts: GrammarOptions) -> str:
    """JSONFunctionStructure.Grammar (marshal -> unmarshal -> converter)."""
    schema = json.loads(_go_json(structure))
    if opts.schema_type == LLAMA31:
        return LLama31SchemaConverter(opts.function_name).grammar(schema, opts)
    return JSONSchemaConverter(opts.prop_order).grammar(schema, opts)


# --------------------------------------------------------------------------- parsing
@dataclass
class FuncCallResult:
    name: str
    arguments: str


def cleanup_llm_result(s: str, fcfg: Optional[dict]) -> str:
    for item in (fcfg or {}).get("replace_llm_results") or []:
        s = re.sub(_go_re(item.get("key", "")), _go_repl(item.get("value", "")), s)
    return s


def parse_text_content(s: str, fcfg: Optional[dict]) -> str:
    for r in (fcfg or {}).get("capture_llm_results") or []:
        m = re.search(_go_re(r), s)
        if m:
            return (m.group(1) if m.groups() else m.group(0)).strip()
    return ""


class JSONTruncated(ValueError):
    """parse.go ParseJSON's non-syntax error: the text ends inside a JSON value (io.ErrUnexpectedEOF)."""

    def __init__(self, msg: str, objs: List[dict]):
        super().__init__(msg)
        self.objs = objs


def _truncated_value(rest: str, e: json.JSONDecodeError) -> bool:
    """Would Go's decoder report unexpected EOF (not a syntax error) on `rest`?  Either the error
    sits at the very end of the input, or what is left is a proper prefix of null / true / false."""
    if e.pos >= len(e.doc):
        return True
    r = rest.strip()
    return bool(r) and any(lit.startswith(r) and lit != r for lit in ("null", "true", "false"))


def parse_json_strict(s: str) -> List[dict]:
    """parse.go ParseJSON including its error: raises JSONTruncated (carrying the objects decoded
    so far) when the text ends inside a value."""
    return _parse_json(s, True)


def parse_json(s: str) -> List[dict]:
    """Tolerant decoder of one or more JSON objects embedded in text (parse.go ParseJSON); the
    callers (ParseFunctionCall) only log ParseJSON's error, so it is swallowed here."""
    return _parse_json(s, False)


def _parse_json(s: str, strict: bool) -> List[dict]:
    objs = []
    dec = json.JSONDecoder()
    off = 0
    n = len(s)
    while off < n:
        while off < n and s[off] in " \t\r\n":
            off += 1
        if off >= n:
            break
        try:
            obj, end = dec.raw_decode(s, off)
            if isinstance(obj, dict):
                objs.append(obj)
            elif isinstance(obj, list):  # parallel calls: [ {...}, {...} ]
                objs.extend(o for o in obj if isinstance(o, dict))
            off = max(end, off + 1)
        except json.JSONDecodeError as e:
            if strict and _truncated_value(s[off:], e):
                raise JSONTruncated(f"unexpected end of JSON input at offset {off}", objs) from e
            off = max(e.pos, off + 1)
    return objs


def _go_re(p: str) -> str:
    # Go RE2 named groups (?P<name>...) are Python-compatible; (?s) etc. are the same
    return p


def _go_repl(v: str) -> str:
    # Go ReplaceAllString expands $1 / ${name}; translate to Python's \1 / \g<name>
    v = v.replace("\\", "\\\\")
    v = re.sub(r"\$\{(\w+)\}", r"\\g<\1>", v)
    return re.sub(r"\$(\d+)", r"\\g<\1>", v)


def parse_function_call(s: str, fcfg: Optional[dict]) -> List[FuncCallResult]:
    fcfg = fcfg or {}
    for item in fcfg.get("replace_function_results") or []:
        s = re.sub(_go_re(item.get("key", "")), _go_repl(item.get("value", "")), s)
    nk = fcfg.get("function_name_key") or DEFAULT_NAME_KEY
    ak = fcfg.get("function_arguments_key") or DEFAULT_ARGS_KEY

    def from_json(texts):
        out = []
        for t in texts:
            for o in parse_json(escape_new_lines(t)):
                if nk not in o or ak not in o:
                    continue
                if not isinstance(o[nk], str):
                    continue
                out.append(FuncCallResult(o[nk], _go_json(o[ak])))
        return out

    llm_results: List[str] = []
    for r in fcfg.get("json_regex_match") or []:
        ms = [m.group(1) for m in re.finditer(_go_re(r), s) if m.groups()]
        if ms:
            llm_results.extend(ms)
            break
    results: List[FuncCallResult] = []
    if fcfg.get("response_regex"):
        for r in fcfg["response_regex"]:
            rx = re.compile(_go_re(r))
            for m in rx.finditer(s):
                d = {k: v for k, v in m.groupdict().items() if v is not None}
                fname = d.get(nk, "")
                if not fname:
                    return results
                results.append(FuncCallResult(fname, d.get(ak, "")))
        return results
    if not llm_results:
        llm_results = [s]
    return from_json(llm_results)
