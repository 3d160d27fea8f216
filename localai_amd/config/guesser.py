"""GGUF-based template guessing (`core/config/guesser.go:33-246`).

When a model config has no template, read the GGUF header, identify the family from the
chat template / architecture / EOS id, and fill templates + stop words (+ repeat penalty)."""
from __future__ import annotations

import logging
import os

log = logging.getLogger("localai_amd.config")

UNKNOWN, LLAMA3, COMMAND_R, PHI3, CHATML, MISTRAL03, GEMMA, DEEPSEEK2 = range(8)

DEFAULTS = {
    GEMMA: {
        "repeat_penalty": 1.0,
        "stopwords": ["<|im_end|>", "<end_of_turn>", "<start_of_turn>"],
        "template": {
            "chat": "{{.Input }}\n<start_of_turn>model\n",
            "chat_message": "<start_of_turn>{{if eq .RoleName \"assistant\" }}model{{else}}{{ .RoleName }}{{end}}\n"
                            "{{ if .Content -}}\n{{.Content -}}\n{{ end -}}<end_of_turn>",
            "completion": "{{.Input}}",
        },
    },
    DEEPSEEK2: {
        "stopwords": ["<｜end▁of▁sentence｜>"],
        "template": {
            "chat_message": "{{if eq .RoleName \"user\" -}}User: {{.Content }}\n{{ end -}}\n"
                            "{{if eq .RoleName \"assistant\" -}}Assistant: {{.Content}}<｜end▁of▁sentence｜>{{end}}\n"
                            "{{if eq .RoleName \"system\" -}}{{.Content}}\n{{end -}}",
            "chat": "{{.Input -}}\nAssistant: ",
        },
    },
    LLAMA3: {
        "stopwords": ["<|eot_id|>"],
        "template": {
            "chat": "<|begin_of_text|>{{.Input }}\n<|start_header_id|>assistant<|end_header_id|>",
            "chat_message": "<|start_header_id|>{{ .RoleName }}<|end_header_id|>\n\n{{.Content }}<|eot_id|>",
        },
    },
    COMMAND_R: {
        "stopwords": ["<|END_OF_TURN_TOKEN|>"],
        "template": {
            "chat": "{{.Input -}}<|START_OF_TURN_TOKEN|><|CHATBOT_TOKEN|>",
            "function": "<|START_OF_TURN_TOKEN|><|SYSTEM_TOKEN|>\nYou are a function calling AI model, you can call "
                        "the following functions:\n## Available Tools\n{{range .Functions}}\n- {\"type\": \"function\", "
                        "\"function\": {\"name\": \"{{.Name}}\", \"description\": \"{{.Description}}\", \"parameters\": "
                        "{{toJson .Parameters}} }}\n{{end}}\nWhen using a tool, reply with JSON, for instance {\"name\": "
                        "\"tool_name\", \"arguments\": {\"param1\": \"value1\", \"param2\": \"value2\"}}\n"
                        "<|END_OF_TURN_TOKEN|><|START_OF_TURN_TOKEN|><|CHATBOT_TOKEN|>{{.Input -}}",
            "chat_message": "{{if eq .RoleName \"user\" -}}\n<|START_OF_TURN_TOKEN|><|USER_TOKEN|>{{.Content}}"
                            "<|END_OF_TURN_TOKEN|>\n{{- else if eq .RoleName \"system\" -}}\n<|START_OF_TURN_TOKEN|>"
                            "<|SYSTEM_TOKEN|>{{.Content}}<|END_OF_TURN_TOKEN|>\n{{- else if eq .RoleName \"assistant\" -}}"
                            "\n<|START_OF_TURN_TOKEN|><|CHATBOT_TOKEN|>{{.Content}}<|END_OF_TURN_TOKEN|>\n"
                            "{{- else if eq .RoleName \"tool\" -}}\n<|START_OF_TURN_TOKEN|><|SYSTEM_TOKEN|>{{.Content}}"
                            "<|END_OF_TURN_TOKEN|>\n{{- else if .FunctionCall -}}\n<|START_OF_TURN_TOKEN|>"
                            "<|CHATBOT_TOKEN|>{{toJson .FunctionCall}}}<|END_OF_TURN_TOKEN|>\n{{- end -}}",
        },
    },
    PHI3: {
        "stopwords": ["<|end|>", "<|endoftext|>"],
        "template": {"chat": "{{.Input}}\n<|assistant|>", "chat_message": "<|{{ .RoleName }}|>\n{{.Content}}<|end|>",
                     "completion": "{{.Input}}"},
    },
    CHATML: {
        "stopwords": ["<|im_end|>", "<dummy32000>", "</s>"],
        "template": {
            "chat": "{{.Input -}}\n<|im_start|>assistant",
            "function": "<|im_start|>system\nYou are a function calling AI model. You are provided with functions to "
                        "execute. You may call one or more functions to assist with the user query. Don't make "
                        "assumptions about what values to plug into functions. Here are the available tools:\n"
                        "{{range .Functions}}\n{'type': 'function', 'function': {'name': '{{.Name}}', 'description': "
                        "'{{.Description}}', 'parameters': {{toJson .Parameters}} }}\n{{end}}\nFor each function call "
                        "return a json object with function name and arguments\n<|im_end|>\n{{.Input -}}\n"
                        "<|im_start|>assistant",
            "chat_message": "<|im_start|>{{ .RoleName }}\n{{ if .FunctionCall -}}\nFunction call:\n"
                            "{{ else if eq .RoleName \"tool\" -}}\nFunction response:\n{{ end -}}\n{{ if .Content -}}\n"
                            "{{.Content }}\n{{ end -}}\n{{ if .FunctionCall -}}\n{{toJson .FunctionCall}}\n{{ end -}}"
                            "<|im_end|>",
        },
    },
    MISTRAL03: {
        "stopwords": ["<|im_end|>", "<dummy32000>", "</tool_call>", "<|eot_id|>", "<|end_of_text|>", "</s>",
                      "[/TOOL_CALLS]", "[/ACTIONS]"],
        "template": {
            "chat": "{{.Input -}}",
            "function": "[AVAILABLE_TOOLS] [{{range .Functions}}{\"type\": \"function\", \"function\": {\"name\": "
                        "\"{{.Name}}\", \"description\": \"{{.Description}}\", \"parameters\": {{toJson .Parameters}} }}"
                        "{{end}} ] [/AVAILABLE_TOOLS]{{.Input }}",
            "chat_message": "{{if eq .RoleName \"user\" -}}\n[INST] {{.Content }} [/INST]\n{{- else if .FunctionCall -}}"
                            "\n[TOOL_CALLS] {{toJson .FunctionCall}} [/TOOL_CALLS]\n{{- else if eq .RoleName \"tool\" -}}"
                            "\n[TOOL_RESULTS] {{.Content}} [/TOOL_RESULTS]\n{{- else -}}\n{{ .Content -}}\n{{ end -}}",
        },
    },
}

KNOWN_TEMPLATES = {
    "{% if messages[0]['role'] == 'system' %}{% set system_message = messages[0]['content'] %}{% endif %}{% if "
    "system_message is defined %}{{ system_message }}{% endif %}{% for message in messages %}{% set content = "
    "message['content'] %}{% if message['role'] == 'user' %}{{ '<|im_start|>user\\n' + content + '<|im_end|>\\n"
    "<|im_start|>assistant\\n' }}{% elif message['role'] == 'assistant' %}{{ content + '<|im_end|>' + '\\n' }}"
    "{% endif %}{% endfor %}": CHATML,
    "{{ bos_token }}{% for message in messages %}{% if (message['role'] == 'user') != (loop.index0 % 2 == 0) %}"
    "{{ raise_exception('Conversation roles must alternate user/assistant/user/assistant/...') }}{% endif %}"
    "{% if message['role'] == 'user' %}{{ '[INST] ' + message['content'] + ' [/INST]' }}{% elif message['role'] == "
    "'assistant' %}{{ message['content'] + eos_token}}{% else %}{{ raise_exception('Only user and assistant roles "
    "are supported!') }}{% endif %}{% endfor %}": MISTRAL03,
}


def identify_family(r) -> int:
    ct = r.kv.get("tokenizer.chat_template") or ""
    if ct and ct in KNOWN_TEMPLATES:
        return KNOWN_TEMPLATES[ct]
    arch = r.architecture
    eos = r.kv.get("tokenizer.ggml.eos_token_id")
    bos = r.kv.get("tokenizer.ggml.bos_token_id")
    name = str(r.kv.get("general.name", "")).lower()
    is_yi = arch == "llama" and bos == 1 and eos == 2
    if arch == "deepseek2":
        return DEEPSEEK2
    if arch.startswith("gemma") or "gemma" in name:
        return GEMMA
    if arch == "llama" and eos == 128009:
        return LLAMA3
    if arch == "command-r" and eos == 255001:
        return COMMAND_R
    if arch == "phi-3":
        return PHI3
    if arch == "qwen2" or is_yi:
        return CHATML
    return UNKNOWN


def guess_defaults_from_file(cfg, model_path: str):
    if os.environ.get("LOCALAI_DISABLE_GUESSING") == "true":
        return
    if not model_path or cfg.has_template():
        return
    path = os.path.join(model_path, cfg.model_file_name())
    if not cfg.model_file_name() or not os.path.isfile(path):
        return
    try:
        from ..gguf import GGUFReader
        r = GGUFReader(path, load_tensors=False)
    except Exception:
        return  # only GGUF files are guessed
    try:
        if not cfg.name:
            cfg.name = str(r.kv.get("general.name", ""))
        fam = identify_family(r)
    finally:
        r.close()
    if fam == UNKNOWN:
        return
    st = DEFAULTS.get(fam)
    if not st:
        return
    cfg.raw["template"] = dict(st["template"])
    if not cfg.stopwords:
        cfg.stopwords = st.get("stopwords", [])
    if not cfg.p("repeat_penalty") and "repeat_penalty" in st:
        cfg.set_p("repeat_penalty", st["repeat_penalty"])
    log.debug("guessed family %s for %s", fam, cfg.name)
