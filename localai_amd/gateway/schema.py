"""Typed request / response models of the HTTP API (reference `core/schema/*.go`: openai.go,
prediction.go, localai.go, jina.go, elevenlabs.go, tokenize.go, transcription.go).

The reference decodes every body into these Go structs with encoding/json, so a field of the
wrong JSON type (a string for `temperature`, an object for `max_tokens`) fails the request with
400 "failed reading parameters from request", while unknown fields are ignored and `null` leaves a
field at its zero value.  The models below reproduce that contract with pydantic (strict scalar
types, every field optional, extra keys allowed) and feed /swagger: each route documents its
body.  Handlers keep working on the validated JSON object (the backend-config merge in
gateway/inference.py reads it as a mapping)."""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Type

from pydantic import BaseModel, ConfigDict, Field, StrictBool, StrictFloat, StrictInt, StrictStr, ValidationError

Num = Optional[StrictFloat | StrictInt]  # Go float64 fields accept JSON integers too


class _Body(BaseModel):
    model_config = ConfigDict(extra="allow", populate_by_name=True)


# ------------------------------------------------------------------ prediction.go
class PredictionOptions(_Body):
    model: Optional[StrictStr] = Field(None, description="model name (config name or model file)")
    language: Optional[StrictStr] = None
    translate: Optional[StrictBool] = None
    n: Optional[StrictInt] = Field(None, description="number of choices")
    top_p: Num = None
    top_k: Optional[StrictInt] = None
    temperature: Num = None
    max_tokens: Optional[StrictInt] = None
    echo: Optional[StrictBool] = None
    batch: Optional[StrictInt] = None
    ignore_eos: Optional[StrictBool] = None
    repeat_penalty: Num = None
    repeat_last_n: Optional[StrictInt] = None
    n_keep: Optional[StrictInt] = None
    frequency_penalty: Num = None
    presence_penalty: Num = None
    tfz: Num = None
    typical_p: Num = None
    seed: Optional[StrictInt] = None
    negative_prompt: Optional[StrictStr] = None
    rope_freq_base: Num = None
    rope_freq_scale: Num = None
    negative_prompt_scale: Num = None
    use_fast_tokenizer: Optional[StrictBool] = None
    clip_skip: Optional[StrictInt] = None
    tokenizer: Optional[StrictStr] = None
    # sampler knobs of the model config (backend_config.go) that requests may also carry
    mirostat: Optional[StrictInt] = None
    mirostat_eta: Num = None
    mirostat_tau: Num = None
    min_p: Num = None
    logit_bias: Optional[Dict[str, StrictFloat | StrictInt]] = None


# ------------------------------------------------------------------ openai.go
class FunctionCall(_Body):
    name: Optional[StrictStr] = None
    arguments: Optional[StrictStr] = None


class ToolCall(_Body):
    index: Optional[StrictInt] = None
    id: Optional[StrictStr] = None
    type: Optional[StrictStr] = None
    function: Optional[FunctionCall] = None


class ContentURL(_Body):
    url: Optional[StrictStr] = None


class Content(_Body):
    type: Optional[StrictStr] = None
    text: Optional[StrictStr] = None
    image_url: Optional[ContentURL | StrictStr] = None
    audio_url: Optional[ContentURL | StrictStr] = None
    video_url: Optional[ContentURL | StrictStr] = None


class Message(_Body):
    role: Optional[StrictStr] = None
    name: Optional[StrictStr] = None
    content: Any = Field(None, description="a string, or a list of {type: text|image_url|audio_url|video_url} parts")
    function_call: Any = None
    tool_calls: Optional[List[ToolCall]] = None


class FunctionDef(_Body):
    name: Optional[StrictStr] = None
    description: Optional[StrictStr] = None
    strict: Optional[StrictBool] = None
    parameters: Optional[Dict[str, Any]] = None


class Tool(_Body):
    type: Optional[StrictStr] = None
    function: Optional[FunctionDef] = None


class OpenAIRequest(PredictionOptions):
    """Body of /v1/chat/completions, /v1/completions, /v1/edits, /v1/embeddings,
    /v1/images/generations (OpenAIRequest in core/schema/openai.go)."""
    file: Optional[StrictStr] = None
    response_format: Any = Field(None, description='"text" | {"type": "json_object"} | '
                                                   '{"type": "json_schema", "json_schema": {...}} | image "url"/"b64_json"')
    size: Optional[StrictStr] = Field(None, description="image size WxH")
    prompt: Any = Field(None, description="a string or a list of strings")
    instruction: Optional[StrictStr] = None
    input: Any = Field(None, description="a string, a list of strings, or token ids")
    stop: Any = Field(None, description="a string or a list of strings")
    messages: Optional[List[Message]] = None
    functions: Optional[List[FunctionDef]] = None
    function_call: Any = None
    tools: Optional[List[Tool]] = None
    tool_choice: Any = None
    stream: Optional[StrictBool] = None
    mode: Optional[StrictInt] = None
    step: Optional[StrictInt] = None
    grammar: Optional[StrictStr] = None
    grammar_json_functions: Optional[Dict[str, Any]] = None
    backend: Optional[StrictStr] = None
    model_base_name: Optional[StrictStr] = None


class OpenAIUsage(_Body):
    prompt_tokens: int = 0
    completion_tokens: int = 0
    total_tokens: int = 0


class Choice(_Body):
    index: int = 0
    finish_reason: Optional[str] = None
    message: Optional[Message] = None
    delta: Optional[Message] = None
    text: Optional[str] = None


class Item(_Body):
    embedding: Optional[List[float]] = None
    index: int = 0
    object: Optional[str] = None
    url: Optional[str] = None
    b64_json: Optional[str] = None


class OpenAIResponse(_Body):
    created: Optional[int] = None
    object: Optional[str] = None
    id: Optional[str] = None
    model: Optional[str] = None
    choices: Optional[List[Choice]] = None
    data: Optional[List[Item]] = None
    usage: OpenAIUsage = OpenAIUsage()


class OpenAIModel(_Body):
    id: str
    object: str = "model"


class ModelsDataResponse(_Body):
    object: str = "list"
    data: List[OpenAIModel] = []


class APIErrorBody(_Body):
    code: Any = None
    message: str
    param: Optional[str] = None
    type: str = ""


class ErrorResponse(_Body):
    error: Optional[APIErrorBody] = None


# ------------------------------------------------------------------ localai.go / jina.go / elevenlabs.go / tokenize.go
class BackendMonitorRequest(_Body):
    model: Optional[StrictStr] = None


class TokenMetricsRequest(_Body):
    model: Optional[StrictStr] = None


class TTSRequest(_Body):
    model: Optional[StrictStr] = Field(None, description="model name or full path")
    input: Optional[StrictStr] = Field(None, description="text input")
    voice: Optional[StrictStr] = Field(None, description="voice audio file or speaker id")
    backend: Optional[StrictStr] = None
    language: Optional[StrictStr] = None


class StoresSet(_Body):
    store: Optional[StrictStr] = None
    keys: Optional[List[List[StrictFloat | StrictInt]]] = None
    values: Optional[List[StrictStr]] = None


class StoresDelete(_Body):
    store: Optional[StrictStr] = None
    keys: Optional[List[List[StrictFloat | StrictInt]]] = None


class StoresGet(_Body):
    store: Optional[StrictStr] = None
    keys: Optional[List[List[StrictFloat | StrictInt]]] = None


class StoresFind(_Body):
    store: Optional[StrictStr] = None
    key: Optional[List[StrictFloat | StrictInt]] = None
    topk: Optional[StrictInt] = None


class JINARerankRequest(_Body):
    model: Optional[StrictStr] = None
    query: Optional[StrictStr] = None
    documents: Optional[List[StrictStr]] = None
    top_n: Optional[StrictInt] = None


class ElevenLabsTTSRequest(_Body):
    text: Optional[StrictStr] = None
    model_id: Optional[StrictStr] = None


class ElevenLabsSoundGenerationRequest(_Body):
    text: Optional[StrictStr] = None
    model_id: Optional[StrictStr] = None
    duration_seconds: Num = None
    prompt_influence: Num = None
    do_sample: Optional[StrictBool] = None


class TokenizeRequest(_Body):
    content: Optional[StrictStr] = None
    model: Optional[StrictStr] = None


class TokenizeResponse(_Body):
    tokens: List[int] = []


class Segment(_Body):
    id: int
    start: float
    end: float
    text: str
    tokens: List[int] = []


class TranscriptionResult(_Body):
    segments: List[Segment] = []
    text: str = ""


# ------------------------------------------------------------------ helpers
class SchemaError(ValueError):
    """A body that does not decode into its request struct (HTTP 400)."""


def validate(model: Type[BaseModel], body: Any) -> Dict[str, Any]:
    """Check a decoded JSON body against `model`; returns the body (a dict) unchanged.  Raises
    SchemaError naming the first offending field, as the reference's 400 does."""
    if not isinstance(body, dict):
        raise SchemaError("failed reading parameters from request: body must be a JSON object")
    try:
        model.model_validate(body)
    except ValidationError as e:
        err = e.errors()[0]
        loc = ".".join(str(x) for x in err.get("loc", ()))
        raise SchemaError(f"failed reading parameters from request: {loc}: {err.get('msg', 'invalid value')}")
    return body


def _inline(node, defs):
    if isinstance(node, dict):
        ref = node.get("$ref")
        if isinstance(ref, str) and ref.startswith("#/$defs/"):
            return _inline(defs[ref[len("#/$defs/"):]], defs)
        return {k: _inline(v, defs) for k, v in node.items() if k != "$defs"}
    if isinstance(node, list):
        return [_inline(v, defs) for v in node]
    return node


def json_schema(model: Type[BaseModel]) -> dict:
    """`model`'s JSON schema with every $ref inlined (no model here is recursive), so it is valid
    anywhere in the OpenAPI document."""
    sch = model.model_json_schema()
    return _inline(sch, sch.get("$defs", {}))


def body_doc(model: Type[BaseModel]) -> dict:
    """`openapi_extra` documenting a route's JSON body with `model` (for /swagger)."""
    return {"requestBody": {"required": True, "content": {"application/json": {"schema": json_schema(model)}}}}
