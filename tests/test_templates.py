"""Go text/template + sprig interpreter.  Vectors: pkg/model/template_test.go (chatML / llama3
chat-message templates) and pkg/templates/multimodal_test.go."""
import pytest

from localai_amd.templates import CHAT_MESSAGE, TemplateCache, render, template_multimodal

CHATML = (
    '<|im_start|>{{if eq .RoleName "assistant"}}assistant{{else if eq .RoleName "system"}}system'
    '{{else if eq .RoleName "tool"}}tool{{else if eq .RoleName "user"}}user{{end}}\n'
    '{{- if .FunctionCall }}\n<tool_call>\n{{- else if eq .RoleName "tool" }}\n<tool_response>\n{{- end }}\n'
    '{{- if .Content}}\n{{.Content }}\n{{- end }}\n'
    '{{- if .FunctionCall}}\n{{toJson .FunctionCall}}\n{{- end }}\n'
    '{{- if .FunctionCall }}\n</tool_call>\n{{- else if eq .RoleName "tool" }}\n</tool_response>\n{{- end }}'
    '<|im_end|>')

LLAMA3 = (
    '<|start_header_id|>{{if eq .RoleName "assistant"}}assistant{{else if eq .RoleName "system"}}system'
    '{{else if eq .RoleName "tool"}}tool{{else if eq .RoleName "user"}}user{{end}}<|end_header_id|>\n\n'
    '{{ if .FunctionCall -}}\nFunction call:\n{{ else if eq .RoleName "tool" -}}\nFunction response:\n{{ end -}}\n'
    '{{ if .Content -}}\n{{.Content -}}\n{{ else if .FunctionCall -}}\n{{ toJson .FunctionCall -}}\n{{ end -}}\n'
    '<|eot_id|>')

GALAXY = "A long time ago in a galaxy far, far away..."


def _data(role, content="", fc=None):
    return {"SystemPrompt": "", "Role": role, "RoleName": role, "Content": content, "FunctionCall": fc,
            "FunctionName": "", "LastMessage": False, "Function": False, "MessageIndex": 0}


CASES = [
    (LLAMA3, _data("user", GALAXY), f"<|start_header_id|>user<|end_header_id|>\n\n{GALAXY}<|eot_id|>"),
    (LLAMA3, _data("assistant", GALAXY), f"<|start_header_id|>assistant<|end_header_id|>\n\n{GALAXY}<|eot_id|>"),
    (LLAMA3, _data("assistant", "", {"function": "test"}),
     '<|start_header_id|>assistant<|end_header_id|>\n\nFunction call:\n{"function":"test"}<|eot_id|>'),
    (LLAMA3, _data("tool", "Response from tool"),
     "<|start_header_id|>tool<|end_header_id|>\n\nFunction response:\nResponse from tool<|eot_id|>"),
    (CHATML, _data("user", GALAXY), f"<|im_start|>user\n{GALAXY}<|im_end|>"),
    (CHATML, _data("assistant", GALAXY), f"<|im_start|>assistant\n{GALAXY}<|im_end|>"),
    (CHATML, _data("assistant", "", {"function": "test"}),
     '<|im_start|>assistant\n<tool_call>\n{"function":"test"}\n</tool_call><|im_end|>'),
    (CHATML, _data("tool", "Response from tool"),
     "<|im_start|>tool\n<tool_response>\nResponse from tool\n</tool_response><|im_end|>"),
]


@pytest.mark.parametrize("tmpl,data,expected", CASES)
def test_chat_message_vectors(tmpl, data, expected):
    assert render(tmpl, data) == expected


def test_template_cache_file_or_inline(tmp_path):
    (tmp_path / "mytpl.tmpl").write_text("X{{.Input}}Y")
    tc = TemplateCache(str(tmp_path))
    assert tc.evaluate(CHAT_MESSAGE, "mytpl", {"Input": "1"}) == "X1Y"
    assert tc.evaluate(CHAT_MESSAGE, "inline {{.Input}}", {"Input": "2"}) == "inline 2"


@pytest.mark.parametrize("src,data,out", [
    ("{{range $i, $x := .L}}{{$i}}={{$x}};{{end}}", {"L": ["a", "b"]}, "0=a;1=b;"),
    ("{{with .A}}{{.B}}{{else}}none{{end}}", {"A": {"B": "b"}}, "b"),
    ("{{with .A}}{{.B}}{{else}}none{{end}}", {"A": None}, "none"),
    ("{{if and .X (not .Y)}}ok{{end}}", {"X": 1, "Y": 0}, "ok"),
    ("{{ .S | upper }} {{ trim \"  z \" }} {{ printf \"%d-%s\" 3 \"q\" }}", {"S": "ab"}, "AB z 3-q"),
    ("{{- /* comment */ -}} a {{- \"b\" }}", {}, "ab"),
    ("{{len .L}} {{index .L 1}} {{.M.k}}", {"L": [1, 2, 3], "M": {"k": "v"}}, "3 2 v"),
    ("{{$t := .T}}{{range .L}}{{$t}}{{.Name}}{{end}}", {"T": "-", "L": [{"Name": "a"}, {"Name": "b"}]}, "-a-b"),
    ("{{ toJson .F }}", {"F": {"b": 1, "a": [True, None]}}, '{"a":[true,null],"b":1}'),
])
def test_go_template_semantics(src, data, out):
    assert render(src, data) == out


def test_multimodal_placeholders():
    assert template_multimodal("[img-{{.ID}}]{{.Text}}", 1, "bar") == "[img-1]bar"
    assert template_multimodal("<image>{{.Text}}", 0, "x") == "<image>x"
