"""localai_amd — an MI355X-native (gfx950 / CDNA4) inference server with LocalAI's
REST API, YAML model-config format and gRPC backend contract.

Layout:
  gateway/   OpenAI/LocalAI-compatible HTTP API (FastAPI)
  config/    YAML model configs, app config, GGUF template guesser
  templates/ Go text/template interpreter (prompt templating)
  functions/ tools/functions -> GBNF grammar, function-call parsing
  grpc/      backend.proto messages + server/client
  engine/    continuous-batching engine (native C++ scheduler/KV manager in native/)
  models/    model families (llama/mistral, mixtral, phi2, llava)
  ops/       hand-written HIP kernels for gfx950 + PyTorch references
  parallel/  tensor/data parallel over RCCL (torch.distributed "nccl")
"""
__version__ = "0.1.0"
