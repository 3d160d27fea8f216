"""HF BERT checkpoints (sentence-transformers encoders, cross-encoder rerankers) on the BERT
engine: embeddings vs `transformers`' BertModel with sentence-transformers mean / CLS pooling, and
the reranker logit vs BertForSequenceClassification -- the library's own forward is the oracle."""
import json

import pytest
import torch
import torch.nn.functional as F

WORDS = ("the a of to and in is it that for on with as was he she they quick brown fox jumps over lazy "
         "dog run runs running model server token kernel memory stream batch hello world").split()


def _vocab():
    v = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"] + WORDS + ["##s", "##ing", "##ed", "##er", "##ly", ",", ".", "!"]
    v += [c for c in "abcdefghijklmnopqrstuvwxyz"] + ["##" + c for c in "abcdefghijklmnopqrstuvwxyz"]
    return list(dict.fromkeys(v))  # no duplicate pieces (real vocabularies have none)


def _write(d, cls_name, pooling_cls=False, seed=0):
    import transformers as tf
    torch.manual_seed(seed)
    vocab = _vocab()
    cfg = tf.BertConfig(vocab_size=len(vocab), hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                        intermediate_size=128, max_position_embeddings=128, num_labels=1)
    m = getattr(tf, cls_name)(cfg).eval()
    with torch.no_grad():
        for n, p in m.named_parameters():
            if p.dim() >= 2:
                p.normal_(0, 0.1)
    m.save_pretrained(d, safe_serialization=True)
    with open(f"{d}/vocab.txt", "w") as f:
        f.write("\n".join(vocab) + "\n")
    if pooling_cls:
        import os
        os.makedirs(f"{d}/1_Pooling", exist_ok=True)
        with open(f"{d}/1_Pooling/config.json", "w") as f:
            json.dump({"pooling_mode_cls_token": True, "pooling_mode_mean_tokens": False}, f)
    return m


def _ids(text):
    from tokenizers import BertWordPieceTokenizer
    return BertWordPieceTokenizer(_VOCAB_FILE[0], lowercase=True).encode(text).ids


_VOCAB_FILE = [None]


@pytest.mark.parametrize("pooling_cls", [False, True])
def test_sentence_embedding_matches_transformers(tmp_path, pooling_cls):
    from localai_amd.models.bert import BertConfig, BertEmbedder
    d = str(tmp_path / "st")
    m = _write(d, "BertModel", pooling_cls)
    _VOCAB_FILE[0] = f"{d}/vocab.txt"
    emb = BertEmbedder(BertConfig(d, "cpu"))
    for text in ("The quick brown fox jumps over the lazy dog.", "hello world, running models!"):
        ids = emb.tokenize(text)
        assert ids == _ids(text), text  # WordPiece parity with the library tokenizer
        with torch.no_grad():
            h = m(torch.tensor([ids])).last_hidden_state[0]
        ref = F.normalize(h[0] if pooling_cls else h.mean(0), dim=0)
        got = torch.tensor(emb.embed([text])[0])
        assert float((got - ref).abs().max()) < 1e-4


def test_cross_encoder_matches_transformers(tmp_path):
    from localai_amd.models.bert import BertConfig, BertEmbedder
    d = str(tmp_path / "ce")
    m = _write(d, "BertForSequenceClassification", seed=1)
    _VOCAB_FILE[0] = f"{d}/vocab.txt"
    emb = BertEmbedder(BertConfig(d, "cpu"))
    assert emb.is_ranker
    from tokenizers import BertWordPieceTokenizer
    q, doc = "quick fox", "the brown fox jumps over the lazy dog"
    enc = BertWordPieceTokenizer(f"{d}/vocab.txt", lowercase=True).encode(q, doc)
    with torch.no_grad():
        ref = float(m(input_ids=torch.tensor([enc.ids]), token_type_ids=torch.tensor([enc.type_ids])).logits[0, 0])
    assert abs(emb.score(q, doc) - ref) < 1e-4
