"""The `backend.Backend` gRPC contract (wire-compatible with the reference's
`backend/backend.proto`), built from descriptors at import time -- no protoc in this image.

Every message, field number, type and the 17 RPCs match the reference file, so external
LocalAI backends (Python/Go/C++ servers generated from that .proto) plug into our gateway,
and our engine worker serves any LocalAI-compatible client.
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PKG = "backend"

# (name, number, type, label) ; type: scalar name | ".backend.Msg" | "enum:.backend.X"
# label: "" | "repeated" | "optional" (proto3 optional) | "map:<valtype>"
_S, _I32, _I64, _U32, _U64, _F, _B, _BY = "string", "int32", "int64", "uint32", "uint64", "float", "bool", "bytes"

MESSAGES = {
    "MetricsRequest": [],
    "MetricsResponse": [("slot_id", 1, _I32), ("prompt_json_for_slot", 2, _S), ("tokens_per_second", 3, _F),
                        ("tokens_generated", 4, _I32), ("prompt_tokens_processed", 5, _I32)],
    "RerankRequest": [("query", 1, _S), ("documents", 2, _S, "repeated"), ("top_n", 3, _I32)],
    "RerankResult": [("usage", 1, ".backend.Usage"), ("results", 2, ".backend.DocumentResult", "repeated")],
    "Usage": [("total_tokens", 1, _I32), ("prompt_tokens", 2, _I32)],
    "DocumentResult": [("index", 1, _I32), ("text", 2, _S), ("relevance_score", 3, _F)],
    "StoresKey": [("Floats", 1, _F, "repeated")],
    "StoresValue": [("Bytes", 1, _BY)],
    "StoresSetOptions": [("Keys", 1, ".backend.StoresKey", "repeated"), ("Values", 2, ".backend.StoresValue", "repeated")],
    "StoresDeleteOptions": [("Keys", 1, ".backend.StoresKey", "repeated")],
    "StoresGetOptions": [("Keys", 1, ".backend.StoresKey", "repeated")],
    "StoresGetResult": [("Keys", 1, ".backend.StoresKey", "repeated"), ("Values", 2, ".backend.StoresValue", "repeated")],
    "StoresFindOptions": [("Key", 1, ".backend.StoresKey"), ("TopK", 2, _I32)],
    "StoresFindResult": [("Keys", 1, ".backend.StoresKey", "repeated"), ("Values", 2, ".backend.StoresValue", "repeated"),
                         ("Similarities", 3, _F, "repeated")],
    "HealthMessage": [],
    "PredictOptions": [
        ("Prompt", 1, _S), ("Seed", 2, _I32), ("Threads", 3, _I32), ("Tokens", 4, _I32), ("TopK", 5, _I32),
        ("Repeat", 6, _I32), ("Batch", 7, _I32), ("NKeep", 8, _I32), ("Temperature", 9, _F), ("Penalty", 10, _F),
        ("F16KV", 11, _B), ("DebugMode", 12, _B), ("StopPrompts", 13, _S, "repeated"), ("IgnoreEOS", 14, _B),
        ("TailFreeSamplingZ", 15, _F), ("TypicalP", 16, _F), ("FrequencyPenalty", 17, _F), ("PresencePenalty", 18, _F),
        ("Mirostat", 19, _I32), ("MirostatETA", 20, _F), ("MirostatTAU", 21, _F), ("PenalizeNL", 22, _B),
        ("LogitBias", 23, _S), ("MLock", 25, _B), ("MMap", 26, _B), ("PromptCacheAll", 27, _B),
        ("PromptCacheRO", 28, _B), ("Grammar", 29, _S), ("MainGPU", 30, _S), ("TensorSplit", 31, _S),
        ("TopP", 32, _F), ("PromptCachePath", 33, _S), ("Debug", 34, _B), ("EmbeddingTokens", 35, _I32, "repeated"),
        ("Embeddings", 36, _S), ("RopeFreqBase", 37, _F), ("RopeFreqScale", 38, _F), ("NegativePromptScale", 39, _F),
        ("NegativePrompt", 40, _S), ("NDraft", 41, _I32), ("Images", 42, _S, "repeated"),
        ("UseTokenizerTemplate", 43, _B), ("Messages", 44, ".backend.Message", "repeated"),
        ("Videos", 45, _S, "repeated"), ("Audios", 46, _S, "repeated"), ("CorrelationId", 47, _S)],
    "Reply": [("message", 1, _BY), ("tokens", 2, _I32), ("prompt_tokens", 3, _I32)],
    "ModelOptions": [
        ("Model", 1, _S), ("ContextSize", 2, _I32), ("Seed", 3, _I32), ("NBatch", 4, _I32), ("F16Memory", 5, _B),
        ("MLock", 6, _B), ("MMap", 7, _B), ("VocabOnly", 8, _B), ("LowVRAM", 9, _B), ("Embeddings", 10, _B),
        ("NUMA", 11, _B), ("NGPULayers", 12, _I32), ("MainGPU", 13, _S), ("TensorSplit", 14, _S),
        ("Threads", 15, _I32), ("LibrarySearchPath", 16, _S), ("RopeFreqBase", 17, _F), ("RopeFreqScale", 18, _F),
        ("RMSNormEps", 19, _F), ("NGQA", 20, _I32), ("ModelFile", 21, _S), ("Device", 22, _S),
        ("UseTriton", 23, _B), ("ModelBaseName", 24, _S), ("UseFastTokenizer", 25, _B), ("PipelineType", 26, _S),
        ("SchedulerType", 27, _S), ("CUDA", 28, _B), ("CFGScale", 29, _F), ("IMG2IMG", 30, _B),
        ("CLIPModel", 31, _S), ("CLIPSubfolder", 32, _S), ("CLIPSkip", 33, _I32), ("ControlNet", 48, _S),
        ("Tokenizer", 34, _S), ("LoraBase", 35, _S), ("LoraAdapter", 36, _S), ("LoraScale", 42, _F),
        ("NoMulMatQ", 37, _B), ("DraftModel", 39, _S), ("AudioPath", 38, _S), ("Quantization", 40, _S),
        ("GPUMemoryUtilization", 50, _F), ("TrustRemoteCode", 51, _B), ("EnforceEager", 52, _B),
        ("SwapSpace", 53, _I32), ("MaxModelLen", 54, _I32), ("TensorParallelSize", 55, _I32), ("MMProj", 41, _S),
        ("RopeScaling", 43, _S), ("YarnExtFactor", 44, _F), ("YarnAttnFactor", 45, _F), ("YarnBetaFast", 46, _F),
        ("YarnBetaSlow", 47, _F), ("Type", 49, _S), ("FlashAttention", 56, _B), ("NoKVOffload", 57, _B)],
    "Result": [("message", 1, _S), ("success", 2, _B)],
    "EmbeddingResult": [("embeddings", 1, _F, "repeated")],
    "TranscriptRequest": [("dst", 2, _S), ("language", 3, _S), ("threads", 4, _U32), ("translate", 5, _B)],
    "TranscriptResult": [("segments", 1, ".backend.TranscriptSegment", "repeated"), ("text", 2, _S)],
    "TranscriptSegment": [("id", 1, _I32), ("start", 2, _I64), ("end", 3, _I64), ("text", 4, _S),
                          ("tokens", 5, _I32, "repeated")],
    "GenerateImageRequest": [("height", 1, _I32), ("width", 2, _I32), ("mode", 3, _I32), ("step", 4, _I32),
                             ("seed", 5, _I32), ("positive_prompt", 6, _S), ("negative_prompt", 7, _S),
                             ("dst", 8, _S), ("src", 9, _S), ("EnableParameters", 10, _S), ("CLIPSkip", 11, _I32)],
    "TTSRequest": [("text", 1, _S), ("model", 2, _S), ("dst", 3, _S), ("voice", 4, _S), ("language", 5, _S, "optional")],
    "SoundGenerationRequest": [("text", 1, _S), ("model", 2, _S), ("dst", 3, _S), ("duration", 4, _F, "optional"),
                               ("temperature", 5, _F, "optional"), ("sample", 6, _B, "optional"),
                               ("src", 7, _S, "optional"), ("src_divisor", 8, _I32, "optional")],
    "TokenizationResponse": [("length", 1, _I32), ("tokens", 2, _I32, "repeated")],
    "MemoryUsageData": [("total", 1, _U64), ("breakdown", 2, _U64, "map:string")],
    "StatusResponse": [("state", 1, "enum:.backend.StatusResponse.State"), ("memory", 2, ".backend.MemoryUsageData")],
    "Message": [("role", 1, _S), ("content", 2, _S)],
}

STATUS_STATES = [("UNINITIALIZED", 0), ("BUSY", 1), ("READY", 2), ("ERROR", -1)]

# (rpc, request, response, server_streaming)
RPCS = [
    ("Health", "HealthMessage", "Reply", False),
    ("Predict", "PredictOptions", "Reply", False),
    ("LoadModel", "ModelOptions", "Result", False),
    ("PredictStream", "PredictOptions", "Reply", True),
    ("Embedding", "PredictOptions", "EmbeddingResult", False),
    ("GenerateImage", "GenerateImageRequest", "Result", False),
    ("AudioTranscription", "TranscriptRequest", "TranscriptResult", False),
    ("TTS", "TTSRequest", "Result", False),
    ("SoundGeneration", "SoundGenerationRequest", "Result", False),
    ("TokenizeString", "PredictOptions", "TokenizationResponse", False),
    ("Status", "HealthMessage", "StatusResponse", False),
    ("StoresSet", "StoresSetOptions", "Result", False),
    ("StoresDelete", "StoresDeleteOptions", "Result", False),
    ("StoresGet", "StoresGetOptions", "StoresGetResult", False),
    ("StoresFind", "StoresFindOptions", "StoresFindResult", False),
    ("Rerank", "RerankRequest", "RerankResult", False),
    ("GetMetrics", "MetricsRequest", "MetricsResponse", False),
]

_FD = descriptor_pb2.FieldDescriptorProto
_SCALARS = {"string": _FD.TYPE_STRING, "int32": _FD.TYPE_INT32, "int64": _FD.TYPE_INT64, "uint32": _FD.TYPE_UINT32,
            "uint64": _FD.TYPE_UINT64, "float": _FD.TYPE_FLOAT, "bool": _FD.TYPE_BOOL, "bytes": _FD.TYPE_BYTES,
            "double": _FD.TYPE_DOUBLE}


def _fill_field(f, name, num, typ, label=""):
    f.name = name
    f.number = num
    f.json_name = name
    if typ.startswith("enum:"):
        f.type = _FD.TYPE_ENUM
        f.type_name = typ[5:]
    elif typ.startswith("."):
        f.type = _FD.TYPE_MESSAGE
        f.type_name = typ
    else:
        f.type = _SCALARS[typ]
    f.label = _FD.LABEL_REPEATED if label == "repeated" else _FD.LABEL_OPTIONAL


def _build_file() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto()
    fd.name = "backend.proto"
    fd.package = PKG
    fd.syntax = "proto3"
    fd.options.go_package = "github.com/go-skynet/LocalAI/pkg/grpc/proto"
    for mname, fields in MESSAGES.items():
        m = fd.message_type.add()
        m.name = mname
        oneof_idx = 0
        for spec in fields:
            name, num, typ = spec[0], spec[1], spec[2]
            label = spec[3] if len(spec) > 3 else ""
            f = m.field.add()
            if label.startswith("map:"):
                entry = m.nested_type.add()
                entry.name = name[0].upper() + name[1:] + "Entry"
                entry.options.map_entry = True
                _fill_field(entry.field.add(), "key", 1, label[4:])
                _fill_field(entry.field.add(), "value", 2, typ)
                _fill_field(f, name, num, f".{PKG}.{mname}.{entry.name}", "repeated")
                continue
            _fill_field(f, name, num, typ, label)
            if label == "optional":
                f.proto3_optional = True
                od = m.oneof_decl.add()
                od.name = "_" + name
                f.oneof_index = oneof_idx
                oneof_idx += 1
        if mname == "StatusResponse":
            e = m.enum_type.add()
            e.name = "State"
            for n, v in STATUS_STATES:
                ev = e.value.add()
                ev.name = n
                ev.number = v
    svc = fd.service.add()
    svc.name = "Backend"
    for rpc, req, resp, stream in RPCS:
        mm = svc.method.add()
        mm.name = rpc
        mm.input_type = f".{PKG}.{req}"
        mm.output_type = f".{PKG}.{resp}"
        mm.server_streaming = stream
    return fd


_POOL = descriptor_pool.DescriptorPool()
FILE = _POOL.Add(_build_file())


def _cls(name):
    return message_factory.GetMessageClass(_POOL.FindMessageTypeByName(f"{PKG}.{name}"))


M = {name: _cls(name) for name in MESSAGES}
globals().update(M)  # backend_pb.PredictOptions, ...

SERVICE = "backend.Backend"


def method_path(rpc: str) -> str:
    return f"/{SERVICE}/{rpc}"


def proto_text() -> str:
    """Render the contract back to .proto text (docs / external backend authors)."""
    lines = ['syntax = "proto3";', "", f"package {PKG};", "", "service Backend {"]
    for rpc, req, resp, stream in RPCS:
        lines.append(f"  rpc {rpc}({req}) returns ({'stream ' if stream else ''}{resp}) {{}}")
    lines.append("}")
    for mname, fields in MESSAGES.items():
        lines += ["", f"message {mname} {{"]
        if mname == "StatusResponse":
            lines.append("  enum State {")
            lines += [f"    {n} = {v};" for n, v in STATUS_STATES]
            lines.append("  }")
        for spec in fields:
            name, num, typ = spec[0], spec[1], spec[2]
            label = spec[3] if len(spec) > 3 else ""
            t = typ.split(".")[-1] if typ.startswith((".", "enum:")) else typ
            if label.startswith("map:"):
                lines.append(f"  map<{label[4:]}, {t}> {name} = {num};")
            else:
                pre = "repeated " if label == "repeated" else ("optional " if label == "optional" else "")
                lines.append(f"  {pre}{t} {name} = {num};")
        lines.append("}")
    return "\n".join(lines) + "\n"
