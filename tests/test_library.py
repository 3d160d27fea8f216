"""Embedded model library: short names resolve to bundled configurations that the config loader
parses (`embedded/embedded.go`, `pkg/startup/model_preload.go:38-56`)."""
import os

from localai_amd import library
from localai_amd.config.loader import BackendConfigLoader
from localai_amd.startup import install_models


def test_short_url_and_library_lookup():
    assert library.model_short_url("phi-2").startswith("github://")
    assert library.model_short_url("no-such") == "no-such"
    assert library.exists_in_library("llama3-instruct") and not library.exists_in_library("nope")


def test_install_embedded_configs(tmp_path):
    errs = install_models([], str(tmp_path), ["llama3-instruct", "mixtral-instruct", "all-minilm-l6-v2",
                                              "llava-1.6-mistral"])
    assert errs == []
    assert len([f for f in os.listdir(tmp_path) if f.endswith(".yaml")]) == 4
    cl = BackendConfigLoader(str(tmp_path))
    cl.load_from_path(str(tmp_path))
    names = {c.name for c in cl.all()}
    assert {"llama3-8b-instruct", "mixtral-instruct", "all-minilm-l6-v2", "llava-1.6-mistral"} <= names
    c = cl.get("llama3-8b-instruct")
    assert "<|eot_id|>" in c.stopwords and c.template.get("chat_message")
    assert cl.get("llava-1.6-mistral").raw["mmproj"].endswith(".gguf")
    assert cl.get("all-minilm-l6-v2").raw["embeddings"]


def test_unknown_name_is_reported(tmp_path):
    errs = install_models([], str(tmp_path), ["definitely-not-a-model"])
    assert len(errs) == 1


def test_library_covers_every_reference_embedded_model():
    """Every embedded/models/*.yaml name of the reference resolves to a loadable config here."""
    import os

    import yaml

    from localai_amd import library
    from localai_amd.config.backend_config import BackendConfig
    ref = "/root/reference/embedded/models"
    names = sorted(f[:-5] for f in os.listdir(ref)) if os.path.isdir(ref) else sorted(library.EMBEDDED)
    assert len(names) >= 27
    for n in names:
        assert library.exists_in_library(n), n
        cfg = BackendConfig(yaml.safe_load(library.resolve_content(n)))
        assert cfg.name and cfg.validate(), n
