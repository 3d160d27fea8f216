"""The per-model YAML configuration (`core/config/backend_config.go:28-549`).

A `BackendConfig` keeps the parsed YAML mapping (so unknown / future keys round-trip) and
exposes the fields the server uses, with the reference's `SetDefaults` (temp 0.9, top_k 40,
top_p 0.95, mirostat 2, ctx 1024 unless the app overrides, ...), `Validate` (no absolute
paths / `..`, backend-name regex), usecase flags and heuristics, and function-call state.
"""
from __future__ import annotations

import copy
import os
import random
import re
from typing import Any, Dict, List, Optional

import yaml

RAND_SEED = -1

FLAG_ANY = 0
FLAG_CHAT = 1 << 0
FLAG_COMPLETION = 1 << 1
FLAG_EDIT = 1 << 2
FLAG_EMBEDDINGS = 1 << 3
FLAG_RERANK = 1 << 4
FLAG_IMAGE = 1 << 5
FLAG_TRANSCRIPT = 1 << 6
FLAG_TTS = 1 << 7
FLAG_SOUND_GENERATION = 1 << 8
FLAG_LLM = FLAG_CHAT & FLAG_COMPLETION & FLAG_EDIT  # (sic: the reference ANDs them -> 0)

USECASE_FLAGS = {"FLAG_ANY": FLAG_ANY, "FLAG_CHAT": FLAG_CHAT, "FLAG_COMPLETION": FLAG_COMPLETION,
                 "FLAG_EDIT": FLAG_EDIT, "FLAG_EMBEDDINGS": FLAG_EMBEDDINGS, "FLAG_RERANK": FLAG_RERANK,
                 "FLAG_IMAGE": FLAG_IMAGE, "FLAG_TRANSCRIPT": FLAG_TRANSCRIPT, "FLAG_TTS": FLAG_TTS,
                 "FLAG_SOUND_GENERATION": FLAG_SOUND_GENERATION, "FLAG_LLM": FLAG_LLM}

_BACKEND_RE = re.compile(r"^[a-zA-Z0-9-_]+$")


def usecases_from_yaml(items: Optional[List[str]]) -> Optional[int]:
    if not items:
        return None
    r = FLAG_ANY
    for s in items:
        r |= USECASE_FLAGS.get("FLAG_" + str(s).upper(), 0)
    return r


def _looks_like_url(s: str) -> bool:
    return any(s.startswith(p) for p in ("http://", "https://", "huggingface://", "hf://", "github:", "oci://",
                                         "ollama://", "file://"))


def _copy_tree(o: Any) -> Any:
    """Deep copy of YAML/JSON-shaped data (dicts, lists, scalars): every request gets a private
    config (request fields override it), so this runs per request -- copy.deepcopy's memo
    bookkeeping cost ~5x more on a gallery-sized config."""
    if isinstance(o, dict):
        return {k: _copy_tree(v) for k, v in o.items()}
    if isinstance(o, list):
        return [_copy_tree(v) for v in o]
    if isinstance(o, (str, int, float, bool)) or o is None:
        return o
    return copy.deepcopy(o)


class BackendConfig:
    def __init__(self, raw: Optional[Dict[str, Any]] = None):
        self.raw: Dict[str, Any] = _copy_tree(raw) if raw else {}
        self.raw.setdefault("parameters", {})
        if self.raw["parameters"] is None:
            self.raw["parameters"] = {}
        self.raw.setdefault("template", {})
        if self.raw["template"] is None:
            self.raw["template"] = {}
        self.prompt_strings: List[str] = []
        self.input_strings: List[str] = []
        self.input_tokens: List[List[int]] = []
        self.function_call_string = ""
        self.function_call_name_string = ""
        self.response_format = ""
        self.response_format_map: Optional[dict] = None
        self.known_usecases = usecases_from_yaml(self.raw.get("known_usecases"))

    # ------------------------------------------------------------------ generic access
    def get(self, key, default=None):
        v = self.raw.get(key)
        return default if v is None else v

    def p(self, key, default=None):
        v = self.raw["parameters"].get(key)
        return default if v is None else v

    def set_p(self, key, value):
        self.raw["parameters"][key] = value

    def copy(self) -> "BackendConfig":
        c = BackendConfig(self.raw)
        c.known_usecases = self.known_usecases
        return c

    # ------------------------------------------------------------------ identity
    @property
    def name(self) -> str:
        return str(self.raw.get("name") or "")

    @name.setter
    def name(self, v):
        self.raw["name"] = v

    @property
    def backend(self) -> str:
        return str(self.raw.get("backend") or "")

    @backend.setter
    def backend(self, v):
        self.raw["backend"] = v

    @property
    def model(self) -> str:
        return str(self.p("model", "") or "")

    @model.setter
    def model(self, v):
        self.set_p("model", v)

    def model_file_name(self) -> str:
        m = self.model
        if _looks_like_url(m):
            return os.path.basename(m.rstrip("/").split("?")[0])
        return m

    def mmproj_file_name(self) -> str:
        m = str(self.raw.get("mmproj") or "")
        if _looks_like_url(m):
            return os.path.basename(m.rstrip("/").split("?")[0])
        return m

    def is_model_url(self) -> bool:
        return _looks_like_url(self.model)

    # ------------------------------------------------------------------ templates
    @property
    def template(self) -> Dict[str, Any]:
        return self.raw["template"]

    def tpl(self, key: str) -> str:
        return str(self.template.get(key) or "")

    def has_template(self) -> bool:
        return bool(self.tpl("completion") or self.tpl("edit") or self.tpl("chat") or self.tpl("chat_message"))

    @property
    def roles(self) -> Dict[str, str]:
        return self.raw.get("roles") or {}

    @property
    def system_prompt(self) -> str:
        return str(self.raw.get("system_prompt") or "")

    @property
    def stopwords(self) -> List[str]:
        return list(self.raw.get("stopwords") or [])

    @stopwords.setter
    def stopwords(self, v):
        self.raw["stopwords"] = list(v)

    @property
    def functions(self) -> Dict[str, Any]:
        return self.raw.get("function") or {}

    @property
    def feature_flags(self) -> Dict[str, Any]:
        return self.raw.get("feature_flags") or {}

    def feature_enabled(self, name: str) -> bool:
        return bool(self.feature_flags.get(name))

    @property
    def embeddings(self) -> bool:
        return bool(self.raw.get("embeddings"))

    @property
    def context_size(self) -> int:
        return int(self.raw.get("context_size") or 0)

    # ------------------------------------------------------------------ functions state
    def should_use_functions(self) -> bool:
        # (sic) reference: (fcs != "none" || fcs == "") || ShouldCallSpecificFunction()
        return (self.function_call_string != "none" or self.function_call_string == "") or \
            self.should_call_specific_function()

    def should_call_specific_function(self) -> bool:
        return len(self.function_call_name_string) > 0

    def function_to_call(self) -> str:
        n = self.function_call_name_string
        if n and n not in ("none", "auto"):
            return n
        return self.function_call_string

    # ------------------------------------------------------------------ defaults / validation
    def set_defaults(self, ctx: int = 0, threads: int = 0, f16: bool = False, debug: bool = False,
                     model_path: str = "", guess: bool = True):
        pr = self.raw["parameters"]
        if pr.get("seed") is None:
            pr["seed"] = RAND_SEED
        if pr.get("top_k") is None:
            pr["top_k"] = 40
        if pr.get("typical_p") is None:
            pr["typical_p"] = 1.0
        if pr.get("tfz") is None:
            pr["tfz"] = 1.0
        if self.raw.get("mmap") is None:
            self.raw["mmap"] = not bool(os.environ.get("XPU"))
        if self.raw.get("mmlock") is None:
            self.raw["mmlock"] = False
        if pr.get("top_p") is None:
            pr["top_p"] = 0.95
        if pr.get("temperature") is None:
            pr["temperature"] = 0.9
        if pr.get("max_tokens") is None:
            pr["max_tokens"] = 0
        if self.raw.get("mirostat") is None:
            self.raw["mirostat"] = 2
        if self.raw.get("mirostat_eta") is None:
            self.raw["mirostat_eta"] = 0.1
        if self.raw.get("mirostat_tau") is None:
            self.raw["mirostat_tau"] = 5.0
        if self.raw.get("gpu_layers") is None:
            self.raw["gpu_layers"] = 99999999
        if self.raw.get("low_vram") is None:
            self.raw["low_vram"] = False
        if self.raw.get("embeddings") is None:
            self.raw["embeddings"] = False
        if not ctx:
            ctx = 1024
        if self.raw.get("context_size") is None:
            self.raw["context_size"] = ctx
        if not threads:
            threads = 4
        if self.raw.get("threads") is None:
            self.raw["threads"] = threads
        if self.raw.get("f16") is None:
            self.raw["f16"] = f16
        if self.raw.get("debug") is None:
            self.raw["debug"] = False
        if debug:
            self.raw["debug"] = True
        if guess:
            from .guesser import guess_defaults_from_file
            guess_defaults_from_file(self, model_path)

    def validate(self) -> bool:
        targets = [self.backend, self.model, str(self.raw.get("mmproj") or "")]
        targets += [str(f.get("filename", "")) for f in (self.raw.get("download_files") or [])]
        for n in targets:
            if not n:
                continue
            if n.startswith(os.sep) or ".." in n:
                return False
        if self.backend:
            return bool(_BACKEND_RE.match(self.backend))
        return True

    # ------------------------------------------------------------------ usecases
    def has_usecases(self, u: int) -> bool:
        if self.known_usecases is not None and (u & self.known_usecases) == u:
            return True
        return self.guess_usecases(u)

    def guess_usecases(self, u: int) -> bool:
        if u & FLAG_CHAT and not (self.tpl("chat") or self.tpl("chat_message")):
            return False
        if u & FLAG_COMPLETION and not self.tpl("completion"):
            return False
        if u & FLAG_EDIT and not self.tpl("edit"):
            return False
        if u & FLAG_EMBEDDINGS and not self.embeddings:
            return False
        if u & FLAG_IMAGE:
            if self.backend not in ("diffusers", "tinydream", "stablediffusion"):
                return False
            if self.backend == "diffusers" and not (self.raw.get("diffusers") or {}).get("pipeline_type"):
                return False
        if u & FLAG_RERANK and self.backend != "rerankers":
            return False
        if u & FLAG_TRANSCRIPT and self.backend != "whisper":
            return False
        if u & FLAG_TTS and self.backend not in ("piper", "transformers-musicgen", "parler-tts"):
            return False
        if u & FLAG_SOUND_GENERATION and self.backend != "transformers-musicgen":
            return False
        return True

    # ------------------------------------------------------------------ misc
    def resolved_seed(self) -> int:
        s = self.p("seed", RAND_SEED)
        if s == RAND_SEED or s is None:
            return random.randint(0, 2 ** 31 - 1)
        return int(s)

    def to_yaml(self) -> str:
        return yaml.safe_dump(self.raw, sort_keys=False, allow_unicode=True)

    def __repr__(self):
        return f"BackendConfig(name={self.name!r}, backend={self.backend!r}, model={self.model!r})"


def load_yaml_configs(text: str) -> List[BackendConfig]:
    data = yaml.safe_load(text)
    if data is None:
        return []
    if isinstance(data, list):
        return [BackendConfig(d or {}) for d in data]
    return [BackendConfig(data)]
