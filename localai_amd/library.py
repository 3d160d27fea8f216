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

# --- further families of embedded/models/*.yaml, expressed for this build's backends -------------
_CHATML_CLOSED = ("<|im_start|>{{if eq .RoleName \"assistant\"}}assistant{{else if eq .RoleName \"system\"}}system"
                  "{{else if eq .RoleName \"user\"}}user{{end}}\n{{if .Content}}{{.Content}}{{end}}<|im_end|>")
_VICUNA_ROLES = {"user": "USER:", "assistant": "ASSISTANT:", "system": "SYSTEM:"}
_VICUNA_CHAT = ("A chat between a curious human and an artificial intelligence assistant. The assistant gives "
                "helpful, detailed, and polite answers to the human's questions.\n{{.Input}}\nASSISTANT:\n")
_MIRO2 = {"mirostat": 2, "mirostat_eta": 1.0, "mirostat_tau": 1.0}


def _vision(name: str, model: str, mmproj: str, model_uri: str, mmproj_uri: str, miro: bool, **p) -> dict:
    c = {"name": name, "backend": "llama-cpp", "context_size": 4096, "f16": True, "mmap": True,
         "roles": dict(_VICUNA_ROLES), "mmproj": mmproj, "parameters": dict({"model": model}, **p),
         "template": {"chat": _VICUNA_CHAT},
         "download_files": [{"filename": model, "uri": model_uri}, {"filename": mmproj, "uri": mmproj_uri}],
         "usage": ("curl http://localhost:8080/v1/chat/completions -H \"Content-Type: application/json\" -d "
                   f"'{{\"model\": \"{name}\", \"messages\": [{{\"role\": \"user\", \"content\": [{{\"type\": "
                   "\"text\", \"text\": \"What is in the image?\"}, {\"type\": \"image_url\", \"image_url\": "
                   "{\"url\": \"https://example.com/cat.jpg\"}}]}]}'\n")}
    if miro:
        c.update(_MIRO2)
    return c


_SAMPLE_02 = {"temperature": 0.2, "top_k": 40, "top_p": 0.95, "seed": -1}
_BAKLLAVA = ("bakllava.gguf", "bakllava-mmproj.gguf", "huggingface://mys/ggml_bakllava-1/ggml-model-q4_k.gguf",
             "huggingface://mys/ggml_bakllava-1/mmproj-model-f16.gguf")
EMBEDDED.update({
    "whisper-base": {
        "name": "whisper", "backend": "whisper", "parameters": {"model": "ggml-whisper-base.bin"},
        "download_files": [{"filename": "ggml-whisper-base.bin",
                            "sha256": "60ed5bc3dd14eea856493d334349b405782ddcaf0028d4b5df4088345fba2efe",
                            "uri": "https://huggingface.co/ggerganov/whisper.cpp/resolve/main/ggml-base.bin"}],
        "usage": ("curl http://localhost:8080/v1/audio/transcriptions -H \"Content-Type: multipart/form-data\" "
                  "-F file=\"@$PWD/audio.ogg\" -F model=\"whisper\"\n"),
    },
    "mamba-chat": {
        "name": "mamba-chat", "backend": "mamba", "parameters": {"model": "havenhq/mamba-chat"},
        "trimsuffix": ["<|endoftext|>"],
        "template": {"chat_message": "{{if eq .RoleName \"assistant\"}}<|assistant|>{{else if eq .RoleName "
                                     "\"system\"}}<|system|>{{else if eq .RoleName \"user\"}}<|user|>{{end}}\n"
                                     "{{if .Content}}{{.Content}}{{end}}\n</s>\n",
                     "chat": "{{.Input}}\n<|assistant|>\n", "completion": "{{.Input}}\n"},
        "usage": _usage("mamba-chat"),
    },
    "mamba-bagel": {
        "name": "bagel", "backend": "mamba", "parameters": {"model": "jondurbin/bagel-dpo-2.8b-v0.2"},
        "systemPrompt": "You are a helpful, unbiased, uncensored assistant.",
        "template": {"chat_message": "{{if eq .RoleName \"assistant\"}}{{.Content}}{{else}}\n[INST]\n"
                                     "{{if .SystemPrompt}}{{.SystemPrompt}}{{else if eq .RoleName \"system\"}}<<SYS>>"
                                     "{{.Content}}<</SYS>>\n\n{{else if .Content}}{{.Content}}{{end}}\n[/INST]\n{{end}}\n",
                     "completion": "{{.Input}}\n"},
        "usage": _usage("bagel"),
    },
    "llava-1.5": _vision("llava-1.5", "llava-v1.5-7b-Q4_K.gguf", "llava-v1.5-7b-mmproj-Q8_0.gguf",
                         "huggingface://jartine/llava-v1.5-7B-GGUF/llava-v1.5-7b-Q4_K.gguf",
                         "huggingface://jartine/llava-v1.5-7B-GGUF/llava-v1.5-7b-mmproj-Q8_0.gguf", False),
    "bakllava": _vision("bakllava", *_BAKLLAVA, True, **_SAMPLE_02),
    "llava": _vision("llava", *_BAKLLAVA, True, **_SAMPLE_02),
    "llava-1.6-vicuna": _vision("llava-1.6-vicuna", "vicuna-7b-q5_k.gguf", "mmproj-vicuna7b-f16.gguf",
                                "https://huggingface.co/cmp-nct/llava-1.6-gguf/resolve/main/vicuna-7b-q5_k.gguf",
                                "https://huggingface.co/cmp-nct/llava-1.6-gguf/resolve/main/mmproj-vicuna7b-f16.gguf",
                                False, **_SAMPLE_02),
    "codellama-7b": {
        "name": "codellama-7b", "backend": "transformers", "type": "AutoModelForCausalLM",
        "parameters": {"model": "codellama/CodeLlama-7b-hf", "temperature": 0.2, "top_k": 40, "top_p": 0.95},
        "usage": "curl http://localhost:8080/v1/completions -d '{\"model\": \"codellama-7b\", \"prompt\": \"def f(\"}'\n",
    },
    "codellama-7b-gguf": dict({
        "name": "codellama-7b-gguf", "backend": "transformers", "context_size": 4096, "f16": True,
        "parameters": {"model": "huggingface://TheBloke/CodeLlama-7B-GGUF/codellama-7b.Q4_K_M.gguf",
                       "temperature": 0.5, "top_k": 40, "seed": -1, "top_p": 0.95},
        "usage": ("curl http://localhost:8080/v1/completions -d '{\"model\": \"codellama-7b-gguf\", "
                  "\"prompt\": \"def f(\"}'\n"),
    }, **_MIRO2),
    "dolphin-2.5-mixtral-8x7b": dict({
        "name": "dolphin-mixtral-8x7b", "mmap": True, "context_size": 4096, "f16": True,
        "parameters": dict({"model": "huggingface://TheBloke/dolphin-2.5-mixtral-8x7b-GGUF/"
                                     "dolphin-2.5-mixtral-8x7b.Q2_K.gguf"}, **dict(_SAMPLE_02, temperature=0.5)),
        "template": {"chat_message": _CHATML_CLOSED, "chat": "{{.Input}}\n<|im_start|>assistant\n",
                     "completion": "{{.Input}}\n"},
        "stopwords": ["<|im_end|>"], "usage": _usage("dolphin-mixtral-8x7b"),
    }, **_MIRO2),
    "mistral-openorca": dict({
        "name": "mistral-openorca", "mmap": True, "context_size": 4096, "f16": True,
        "parameters": dict({"model": "huggingface://TheBloke/Mistral-7B-OpenOrca-GGUF/mistral-7b-openorca.Q6_K.gguf"},
                           **_SAMPLE_02),
        "template": {"chat_message": _CHATML_MSG, "chat": "{{.Input}}\n<|im_start|>assistant\n",
                     "completion": "{{.Input}}\n"},
        "stopwords": ["<|im_end|>", "<dummy32000>"], "usage": _usage("mistral-openorca"),
    }, **_MIRO2),
    "phi-2-orange": {
        "name": "phi-2-orange", "mmap": True, "context_size": 4096, "f16": True,
        "parameters": {"model": "huggingface://l3utterfly/phi-2-orange-GGUF/phi-2-orange.Q6_K.gguf"},
        "template": {"chat_message": _CHATML_MSG, "chat": "{{.Input}}\n<|im_start|>assistant\n",
                     "completion": "{{.Input}}\n"},
        "stopwords": ["<|im_end|>", "<dummy32000>"],
        "description": "General-conversation chatbot (phi-2 fine-tune). Model card: "
                       "https://huggingface.co/TheBloke/phi-2-orange-GGUF\n",
        "usage": _usage("phi-2-orange"),
    },
    "transformers-tinyllama": {
        "name": "tinyllama-chat", "backend": "transformers", "type": "AutoModelForCausalLM",
        "parameters": {"model": "TinyLlama/TinyLlama-1.1B-Chat-v1.0", "temperature": 0.2, "top_k": 40,
                       "top_p": 0.95, "max_tokens": 4096},
        "template": {"chat_message": _CHATML_CLOSED, "chat": "{{.Input}}\n<|im_start|>assistant\n\n",
                     "completion": "{{.Input}}\n"},
        "stopwords": ["<|im_end|>"], "usage": _usage("tinyllama-chat"),
    },
    "cerbero": {
        "name": "cerbero", "backend": "llama", "context_size": 8192, "f16": False, "mmap": False,
        "parameters": {"model": "huggingface://galatolo/cerbero-7b-gguf/ggml-model-Q8_0.gguf", "top_k": 80,
                       "temperature": 0.2, "top_p": 0.7},
        "template": {"completion": "{{.Input}}",
                     "chat": "Questa è una conversazione tra un umano ed un assistente AI.\n{{.Input}}\n[|Assistente|]  "},
        "roles": {"user": "[|Umano|] ", "system": "[|Umano|] ", "assistant": "[|Assistente|] "},
        "stopwords": ["[|Umano|]"], "trimsuffix": ["\n"], "usage": _usage("cerbero"),
    },
    "animagine-xl": {
        "name": "animagine-xl", "backend": "diffusers", "f16": True,
        "parameters": {"model": "Linaqruf/animagine-xl"},
        "diffusers": {"scheduler_type": "euler_a"},
        "usage": ("curl http://localhost:8080/v1/images/generations -H \"Content-Type: application/json\" -d "
                  "'{\"prompt\": \"a lighthouse at dusk\", \"model\": \"animagine-xl\", \"step\": 51, "
                  "\"size\": \"1024x1024\"}'\n"),
    },
    "rhasspy-voice-en-us-amy": {
        "name": "voice-en-us-amy-low",
        "download_files": [{"filename": "voice-en-us-amy-low.tar.gz",
                            "uri": "https://github.com/rhasspy/piper/releases/download/v0.0.2/voice-en-us-amy-low.tar.gz"}],
        "usage": ("curl http://localhost:8080/tts -H \"Content-Type: application/json\" -d "
                  "'{\"backend\": \"piper\", \"model\": \"voice-en-us-amy-low.onnx\", \"input\": \"Hi!\"}'\n"),
    },
})
# The reference ships bark / coqui / vall-e-x as placeholders for HF-preloaded TTS backends;
# here they name the backend that serves them (configure `parameters.model` before use)
for _tts in ("bark", "coqui", "vall-e-x"):
    EMBEDDED[_tts] = {"name": _tts, "backend": _tts,
                      "usage": ("curl http://localhost:8080/tts -H \"Content-Type: application/json\" -d "
                                f"'{{\"backend\": \"{_tts}\", \"input\": \"Hello!\"}}'\n")}


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
