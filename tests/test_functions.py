"""Function calling: JSON-schema -> GBNF conversion and LLM-output parsing.
Vectors: pkg/functions/grammars/json_schema_test.go, pkg/functions/parse_test.go."""
import json

from localai_amd import functions as fn

SCHEMA1 = {"oneOf": [
    {"type": "object", "properties": {"function": {"const": "create_event"}, "arguments": {
        "type": "object", "properties": {"title": {"type": "string"}, "date": {"type": "string"},
                                         "time": {"type": "string"}}}}},
    {"type": "object", "properties": {"function": {"const": "search"}, "arguments": {
        "type": "object", "properties": {"query": {"type": "string"}}}}},
]}

EXPECTED1 = [
    'root-0-function ::= "\\"create_event\\""',
    'root-0 ::= "{" space "\\"arguments\\"" space ":" space root-0-arguments "," space "\\"function\\"" space ":" '
    'space root-0-function "}" space',
    'root-1-arguments ::= "{" space "\\"query\\"" space ":" space string "}" space',
    "root ::= root-0 | root-1",
    'space ::= " "?',
    'root-0-arguments ::= "{" space "\\"date\\"" space ":" space string "," space "\\"time\\"" space ":" space '
    'string "," space "\\"title\\"" space ":" space string "}" space',
    'root-1 ::= "{" space "\\"arguments\\"" space ":" space root-1-arguments "," space "\\"function\\"" space ":" '
    'space root-1-function "}" space',
    'root-1-function ::= "\\"search\\""',
]


def test_json_schema_grammar_vector():
    g = fn.JSONSchemaConverter("").grammar(SCHEMA1, fn.GrammarOptions())
    for line in EXPECTED1:
        assert line in g, line
    assert "freestring ::=" in g and 'string ::= "\\"" (' in g


def test_maybe_array_and_prefix():
    g = fn.JSONSchemaConverter("").grammar(SCHEMA1, fn.GrammarOptions(maybe_array=True))
    assert "realvalue ::= root-0 | root-1" in g
    assert "root ::= arr | realvalue" in g
    g2 = fn.JSONSchemaConverter("").grammar(SCHEMA1, fn.GrammarOptions(prefix="suffix"))
    assert 'root ::= "suffix" realvalue' in g2 and "realvalue ::= root-0 | root-1" in g2


def test_tools_structure_grammar():
    funcs = [{"name": "get_weather", "description": "w",
              "parameters": {"type": "object", "properties": {"city": {"type": "string"}}}}]
    js = fn.to_json_structure(funcs, "", "")
    g = fn.structure_grammar(js, fn.grammar_options({}))
    assert '"\\"get_weather\\""' in g
    assert g.count("::=") >= 5


def test_parse_function_call_json():
    r = fn.parse_function_call('{"name": "add", "arguments": {"x": 5, "y": 3}}', {})
    assert [(x.name, x.arguments) for x in r] == [("add", '{"x":5,"y":3}')]


def test_parse_function_call_regex():
    r = fn.parse_function_call('add({"x":5,"y":3})', {"response_regex": [r"(?P<name>\w+)\s*\((?P<arguments>.*)\)"]})
    assert [(x.name, x.arguments) for x in r] == [("add", '{"x":5,"y":3}')]
    r = fn.parse_function_call('add({"x":5,"y":3})', {"response_regex": [r"(?P<function>\w+)\s*\((?P<arguments>.*)\)"],
                                                       "function_name_key": "function"})
    assert [(x.name, x.arguments) for x in r] == [("add", '{"x":5,"y":3}')]


def test_parse_invalid_and_parallel():
    assert fn.parse_function_call("", {}) == []
    assert fn.parse_function_call("invalid input", {}) == []
    r = fn.parse_function_call('[{"name": "add", "arguments": {"x": 5, "y": 3}}, '
                               '{"name": "subtract", "arguments": {"x": 10, "y": 7}}]', {})
    assert [(x.name, x.arguments) for x in r] == [("add", '{"x":5,"y":3}'), ("subtract", '{"x":10,"y":7}')]


def test_parse_name_key_and_json_regex_match():
    r = fn.parse_function_call('{"function": "add", "arguments": {"x": 5, "y": 3}}', {"function_name_key": "function"})
    assert [(x.name, x.arguments) for x in r] == [("add", '{"x":5,"y":3}')]
    s = '<tool_call>{"name": "add", "arguments": {"x": 5, "y": 3}}</tool_call>'
    r = fn.parse_function_call(s, {"json_regex_match": [r"(?s)<tool_call>(.*?)</tool_call>"]})
    assert [(x.name, x.arguments) for x in r] == [("add", '{"x":5,"y":3}')]


def test_replace_results_and_cleanup():
    cfg = {"replace_function_results": [{"key": "'", "value": '"'}]}
    r = fn.parse_function_call("{'name': 'add', 'arguments': {'x': 5}}", cfg)
    assert r and r[0].name == "add" and json.loads(r[0].arguments) == {"x": 5}
    out = fn.cleanup_llm_result("xx<think>a</think>yy", {"replace_llm_results": [{"key": "(?s)<think>.*</think>",
                                                                                    "value": ""}]})
    assert out == "xxyy"


def test_parse_text_content_capture():
    s = "Some text <tool_call>{}</tool_call>"
    assert fn.parse_text_content(s, {"capture_llm_results": [r"(?s)^(.*?)<tool_call>"]}) == "Some text"
