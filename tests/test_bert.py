"""BERT sentence-embedding engine (reference: bert-embeddings backend / sentencetransformers)."""
import asyncio
import math

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


def _ref_rank_logit(e, query, doc):
    """Plain fp32 PyTorch cross-encoder forward (the numerics oracle for BertEmbedder.score)."""
    import torch.nn.functional as F
    q = e.tok.encode(query)
    d = e.tok.encode(doc, add_special=False) + [e.tok.sep]
    ids = torch.tensor(q + d)
    types = torch.tensor([0] * len(q) + [1] * len(d))
    D, H = e.dim, e.heads
    n = len(ids)
    x = e.tok_emb.float()[ids] + e.pos_emb.float()[:n] + e.type_emb.float()[types]
    x = F.layer_norm(x, (D,), e.emb_ln[0], e.emb_ln[1], e.eps)
    for ly in e.layers:
        qkv = x @ ly["qkv"].float().t() + ly["qkv_b"]
        qh, kh, vh = qkv.view(n, 3, H, D // H).permute(1, 2, 0, 3)
        att = torch.softmax(qh @ kh.transpose(-1, -2) / math.sqrt(D // H), -1) @ vh
        a = att.transpose(0, 1).reshape(n, D) @ ly["o"].float().t() + ly["o_b"]
        x = F.layer_norm(x + a, (D,), ly["ln1"][0], ly["ln1"][1], e.eps)
        h = F.gelu(x @ ly["up"].float().t() + ly["up_b"]) @ ly["down"].float().t() + ly["down_b"]
        x = F.layer_norm(x + h, (D,), ly["ln2"][0], ly["ln2"][1], e.eps)
    c = torch.tanh(x[0] @ e.cls_w.t() + e.cls_b)
    return float(c @ e.cls_out_w.reshape(-1) + e.cls_out_b.reshape(-1)[0])


def test_cross_encoder_rerank(tmp_path):
    p = synth.write_bert(str(tmp_path / "rank.gguf"), dim=64, n_layer=2, heads=4, ffn=128, ranker=True, std=0.2)
    e = BertEmbedder(BertConfig(p, "cpu"))
    assert e.is_ranker and e.pooling == 4
    docs = ["the quick brown fox", "gpu kernel memory stream", "hello world"]
    rel = e.rerank("quick fox", docs)
    assert len(rel) == 3 and all(0.0 < r < 1.0 for r in rel)
    for d, r in zip(docs, rel):
        ref = _ref_rank_logit(e, "quick fox", d)
        assert abs(e.score("quick fox", d) - ref) < 1e-4
        assert abs(r - 1.0 / (1.0 + math.exp(-ref))) < 1e-5
    # segment ids matter: the pair encoding is not the concatenated single-segment text
    assert len(set(round(r, 6) for r in rel)) == 3


def test_servicer_rerank_uses_cross_encoder(tmp_path):
    from localai_amd.grpc import backend_pb as pb
    from localai_amd.grpc.servicer import EngineServicer
    p = synth.write_bert(str(tmp_path / "rank.gguf"), dim=64, n_layer=1, heads=4, ffn=128, ranker=True, std=0.2)
    sv = EngineServicer(device="cpu")
    docs = ["the quick brown fox", "gpu kernel memory stream", "hello world"]

    async def go():
        r = await sv.LoadModel(pb.ModelOptions(ModelFile=p, ContextSize=128))
        assert r.success, r.message
        return await sv.Rerank(pb.RerankRequest(query="quick fox", documents=docs, top_n=2))
    res = asyncio.run(go())
    assert len(res.results) == 2
    expect = sorted(range(3), key=lambda i: -sv.engine.rerank("quick fox", docs)[i])[:2]
    assert [r.index for r in res.results] == expect
    assert res.results[0].relevance_score >= res.results[1].relevance_score
