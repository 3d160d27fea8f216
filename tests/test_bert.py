"""BERT sentence-embedding engine (reference: bert-embeddings backend / sentencetransformers)."""
import asyncio

import torch

from localai_amd.models import synth
from localai_amd.models.bert import BertConfig, BertEmbedder, WordPiece


def test_wordpiece_rules():
    toks = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "▁hello", "▁wor", "ld", "▁!", "▁a"]
    wp = WordPiece(toks, 1, 2, 3)
    assert wp.encode("Hello world!") == [2, 4, 5, 6, 7, 3]
    assert wp.encode("zzz") == [2, 1, 3]
    assert WordPiece.basic("Héllo,  World") == ["hello", ",", "world"]


def test_bert_embeddings(tmp_path):
    p = synth.write_bert(str(tmp_path / "bert.gguf"), dim=64, n_layer=2, heads=4, ffn=128)
    e = BertEmbedder(BertConfig(p, "cpu"))
    a, b, c = e.embed(["the quick brown fox", "the quick brown fox", "gpu kernel memory"])
    assert len(a) == 64 and abs(sum(x * x for x in a) - 1) < 1e-4
    assert a == b and a != c


def test_servicer_loads_bert_and_embeds(tmp_path):
    from localai_amd.grpc import backend_pb as pb
    from localai_amd.grpc.servicer import EngineServicer
    p = synth.write_bert(str(tmp_path / "bert.gguf"), dim=64, n_layer=1, heads=4, ffn=128)
    sv = EngineServicer(device="cpu")

    async def go():
        r = await sv.LoadModel(pb.ModelOptions(ModelFile=p, ContextSize=128))
        assert r.success, r.message
        res = await sv.Embedding(pb.PredictOptions(Embeddings="hello world"))
        return list(res.embeddings)
    v = asyncio.run(go())
    assert len(v) == 64 and torch.isfinite(torch.tensor(v)).all()
