"""Embedded model library (`embedded/embedded.go`, `embedded/model_library.yaml`,
`embedded/models/*.yaml`): short names that expand to a model URL, and complete model
configurations shipped with the package.  `local-ai run <name>` / `--models <name>` resolves a
name here before trying URLs, local files and galleries (`pkg/startup/model_preload.go:21-140`).

The bundled configurations cover the families this build serves natively on MI355X: Llama-3
(chat + tool calling), Mixtral MoE, Mistral/Hermes chatml, Phi-2, TinyLlama, LLaVA-1.6 (vision)
and BERT sentence embeddings.  Files are fetched on first load through the downloader
(huggingface:// URIs); with no network they can be dropped into the models directory by hand.
"""
from __future__ import annotations

from typing import Dict, Optional

import yaml

# name -> URL of a model file or of a YAML configuration
SHORTENERS: Dict[str, str] = {
    "phi-2": "github://mudler/LocalAI/examples/configurations/phi-2.yaml@master",
}

_LLAMA3_MSG = """<|start_header_id|>{{if eq .RoleName "assistant"}}assistant{{else if eq .RoleName "system"}}system{{else if eq .RoleName "tool"}}tool{{else}}user{{end}}<|end_header_id|>

{{ if .FunctionCall -}}
Function call:
{{ else if eq .RoleName "tool" -}}
Function response:
{{ end -}}
{{ if .Content -}}
{{.Content -}}
{{ else if .FunctionCall -}}
{{ toJson .FunctionCall -}}
{{ end -}}
<|eot_id|>"""

_CHATML_MSG = """<|im_start|>{{if eq .RoleName "assistant"}}assistant{{else if eq .RoleName "system"}}system{{else if eq .RoleName "tool"}}tool{{else}}user{{end}}
{{if .Content}}{{.Content}}{{end}}{{if .FunctionCall}}{{toJson .FunctionCall}}{{end}}
<|im_end|>"""

_TOOLS_SYS = """You can call functions. The available tools, as JSON schemas:
{{range .Functions}}
{"name": "{{.Name}}", "description": "{{.Description}}", "parameters": {{toJson .Parameters}}}
{{end}}
Answer with one JSON object {"name": <tool name>, "arguments": <object>} per call."""


def _usage(name: str) -> str:
    return ("curl http://localhost:8080/v1/chat/completions -H \"Content-Type: application/json\" "
            f"-d '{{\"model\": \"{name}\", \"messages\": [{{\"role\": \"user\", \"content\": \"Hello\"}}]}}'\n")


EMBEDDED: Dict[str, dict] = {
    "llama3-instruct": {
        "name": "llama3-8b-instruct",
        "mmap": True,
        "parameters": {"model": "huggingface://QuantFactory/Meta-Llama-3-8B-Instruct-GGUF/"
                                "Meta-Llama-3-8B-Instruct.Q4_K_M.gguf"},
        "template": {
            "chat_message": _LLAMA3_MSG,
            "function": "<|start_header_id|>system<|end_header_id|>\n\n" + _TOOLS_SYS
                        + "<|eot_id|><|start_header_id|>assistant<|end_header_id|>\nFunction call:\n",
            "chat": "<|begin_of_text|>{{.Input }}\n<|start_header_id|>assistant<|end_header_id|>\n",
            "completion": "{{.Input}}",
        },
        "context_size": 8192,
        "f16": True,
        "stopwords": ["<|eot_id|>", "<|end_of_text|>"],
        "usage": _usage("llama3-8b-instruct"),
    },
    "mixtral-instruct": {
        "name": "mixtral-instruct",
        "mmap": True,
        "parameters": {"model": "huggingface://TheBloke/Mixtral-8x7B-Instruct-v0.1-GGUF/"
                                "mixtral-8x7b-instruct-v0.1.Q4_K_M.gguf"},
        "template": {
            "chat": "{{.Input}}",
            "chat_message": "{{if eq .RoleName \"user\"}}[INST] {{.Content}} [/INST]{{else}}{{.Content}}</s>{{end}}",
            "completion": "[INST] {{.Input}} [/INST]",
        },
        "context_size": 4096,
        "f16": True,
        "stopwords": ["</s>", "[/INST]"],
        "usage": _usage("mixtral-instruct"),
    },
    "hermes-2-pro-mistral": {
        "name": "hermes-2-pro-mistral",
        "mmap": True,
        "parameters": {"model": "huggingface://NousResearch/Hermes-2-Pro-Mistral-7B-GGUF/"
                                "Hermes-2-Pro-Mistral-7B.Q4_K_M.gguf"},
        "template": {
            "chat_message": _CHATML_MSG,
            "function": "<|im_start|>system\n" + _TOOLS_SYS + "<|im_end|>\n{{.Input -}}\n<|im_start|>assistant\n",
            "chat": "{{.Input -}}\n<|im_start|>assistant\n",
            "completion": "{{.Input}}",
        },
        "context_size": 4096,
        "f16": True,
        "stopwords": ["<|im_end|>", "<dummy32000>", "</tool_call>"],
        "usage": _usage("hermes-2-pro-mistral"),
    },
    "phi-2-chat": {
        "name": "phi-2-chat",
        "mmap": True,
        "parameters": {"model": "huggingface://TheBloke/phi-2-GGUF/phi-2.Q8_0.gguf"},
        "template": {"chat_message": _CHATML_MSG, "chat": "{{.Input}}\n<|im_start|>assistant\n",
                     "completion": "{{.Input}}"},
        "context_size": 2048,
        "f16": True,
        "stopwords": ["<|im_end|>", "<|endoftext|>"],
        "usage": _usage("phi-2-chat"),
    },
    "tinyllama-chat": {
        "name": "tinyllama-chat",
        "mmap": True,
        "parameters": {"model": "huggingface://TheBloke/TinyLlama-1.1B-Chat-v1.0-GGUF/"
                                "tinyllama-1.1b-chat-v1.0.Q8_0.gguf"},
        "template": {"chat_message": "<|{{.RoleName}}|>\n{{.Content}}</s>",
                     "chat": "{{.Input}}\n<|assistant|>\n", "completion": "{{.Input}}"},
        "context_size": 2048,
        "f16": True,
        "stopwords": ["</s>"],
        "usage": _usage("tinyllama-chat"),
    },
    "llava-1.6-mistral": {
        "name": "llava-1.6-mistral",
        "mmap": True,
        "mmproj": "llava-v1.6-mistral-7b-mmproj-f16.gguf",
        "parameters": {"model": "llava-v1.6-mistral-7b.Q5_K_M.gguf", "temperature": 0.2},
        "template": {"chat": "[INST] {{.Input}} [/INST]",
                     "chat_message": "{{if eq .RoleName \"user\"}}{{.Content}}{{else}}{{.Content}}</s>{{end}}"},
        "context_size": 4096,
        "f16": True,
        "stopwords": ["</s>"],
        "download_files": [
            {"filename": "llava-v1.6-mistral-7b.Q5_K_M.gguf",
             "uri": "huggingface://cjpais/llava-1.6-mistral-7b-gguf/llava-v1.6-mistral-7b.Q5_K_M.gguf"},
            {"filename": "llava-v1.6-mistral-7b-mmproj-f16.gguf",
             "uri": "huggingface://cjpais/llava-1.6-mistral-7b-gguf/mmproj-model-f16.gguf"},
        ],
        "usage": ("curl http://localhost:8080/v1/chat/completions -H \"Content-Type: application/json\" -d "
                  "'{\"model\": \"llava-1.6-mistral\", \"messages\": [{\"role\": \"user\", \"content\": "
                  "[{\"type\": \"text\", \"text\": \"What is in the image?\"}, {\"type\": \"image_url\", "
                  "\"image_url\": {\"url\": \"https://example.com/cat.jpg\"}}]}]}'\n"),
    },
    "all-minilm-l6-v2": {
        "name": "all-minilm-l6-v2",
        "backend": "bert-embeddings",
        "embeddings": True,
        "parameters": {"model": "huggingface://leliuga/all-MiniLM-L6-v2-GGUF/all-MiniLM-L6-v2.F16.gguf"},
        "usage": ("curl http://localhost:8080/v1/embeddings -H \"Content-Type: application/json\" "
                  "-d '{\"input\": \"Your text string goes here\", \"model\": \"all-minilm-l6-v2\"}'\n"),
    },
}
EMBEDDED["bert-cpp"] = dict(EMBEDDED["all-minilm-l6-v2"], name="bert-cpp-minilm-v6")


def model_short_url(s: str) -> str:
    """ModelShortURL."""
    return SHORTENERS.get(s, s)


def exists_in_library(s: str) -> bool:
    return s in EMBEDDED


def resolve_content(s: str) -> bytes:
    if s not in EMBEDDED:
        raise KeyError(f"cannot find model {s}")
    return yaml.safe_dump(EMBEDDED[s], sort_keys=False, allow_unicode=True).encode()


def remote_library_shorteners(url: str, base_path: str) -> Dict[str, str]:
    """GetRemoteLibraryShorteners: a YAML map name -> URL fetched through the downloader."""
    from .utils.downloader import read_uri
    data = yaml.safe_load(read_uri(url, base_path)) or {}
    if not isinstance(data, dict):
        raise ValueError("remote library is not a name -> URL map")
    return {str(k): str(v) for k, v in data.items()}


def list_models() -> Dict[str, Optional[str]]:
    """Every resolvable short name with a one-line description (for `models list`)."""
    out: Dict[str, Optional[str]] = {k: f"config ({v.get('name', k)})" for k, v in EMBEDDED.items()}
    out.update({k: v for k, v in SHORTENERS.items()})
    return out
