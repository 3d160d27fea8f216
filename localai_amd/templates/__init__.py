"""Prompt templating (Go text/template + sprig compatible) and the template cache
(`pkg/templates/cache.go`, `pkg/model/template.go`, `pkg/templates/multimodal.go`)."""
from __future__ import annotations

import os
import threading
from typing import Any, Dict

from .gotemplate import NO_VALUE, Template, TemplateError, go_str, render, truth  # noqa: F401

CHAT_PROMPT, CHAT_MESSAGE, COMPLETION_PROMPT, EDIT_PROMPT, FUNCTIONS_PROMPT = range(5)


class TemplateCache:
    """Template = `<models_dir>/<name>.tmpl` if that file exists, otherwise the name string
    itself is the template source (cache.go:66-103).  Parsed templates are cached per type."""

    def __init__(self, templates_path: str):
        self.path = templates_path
        self._lock = threading.Lock()
        self._cache: Dict[tuple, Template] = {}

    def _load(self, ttype: int, name: str) -> Template:
        key = (ttype, name)
        t = self._cache.get(key)
        if t is not None:
            return t
        src = name
        fname = f"{name}.tmpl"
        if self.path and len(fname) < 256 and "\n" not in fname:
            full = os.path.realpath(os.path.join(self.path, fname))
            root = os.path.realpath(self.path)
            if full.startswith(root + os.sep) and os.path.isfile(full):
                with open(full, "r", encoding="utf-8") as f:
                    src = f.read()
        t = Template(src)
        self._cache[key] = t
        return t

    def evaluate(self, ttype: int, name: str, data: Any) -> str:
        with self._lock:
            t = self._load(ttype, name)
        return t.execute(data)

    def exists(self, name: str) -> bool:
        return bool(self.path) and os.path.isfile(os.path.join(self.path, name))


def template_multimodal(tmpl: str, idx: int, text: str) -> str:
    return Template(tmpl).execute({"ID": idx, "Text": text})
