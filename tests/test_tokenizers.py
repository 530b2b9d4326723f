"""Native C++ tokenizers vs HuggingFace ``tokenizers`` on the same vocabulary files (trained
here on a local corpus: the real GPT-2/BERT vocab files are not available offline)."""
import os

import pytest

from distributed_lms_raft_llm_amd.tokenizer import GPT2BPE, BertWordPiece

CORPUS = [
    "You are an intelligent assistant. Answer the following question in detail:",
    "Question: How does Raft elect a leader when the old one crashes?",
    "Answer: Followers time out, become candidates, request votes; a majority wins the term.",
    "It's the leader's job to replicate log entries; they'll be committed once stored on a quorum.",
    "Numbers like 2024, 3.14159 and 1e-9 appear   with   odd   spacing\nand new lines\t\ttabs.",
    "Unicode: naïve café résumé — “quotes” ünïcödé 東京",
    "def f(x):\n    return x ** 2  # comment!!! ???",
] * 20

SAMPLES = CORPUS[:7] + ["", " ", "  leading spaces", "trailing   ", "a'b 're 've 'll 'd 's 't 'm", "X" * 300,
                        "emoji 🚀 and symbols <>[]{}", "\n\n\nmany\n\n newlines"]


@pytest.fixture(scope="module")
def bpe_files(tmp_path_factory):
    tk = pytest.importorskip("tokenizers")
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers

    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(vocab_size=1200, initial_alphabet=pre_tokenizers.ByteLevel.alphabet(),
                                  show_progress=False)
    tok.train_from_iterator(CORPUS, trainer)
    d = tmp_path_factory.mktemp("bpe")
    tok.model.save(str(d))
    return tok, str(d / "vocab.json"), str(d / "merges.txt")


def test_bpe_matches_hf_on_same_files(bpe_files):
    hf, vocab, merges = bpe_files
    ours = GPT2BPE(vocab, merges, eos_token_id=10 ** 6)
    assert not ours.synthetic
    for s in SAMPLES:
        ref = hf.encode(s).ids
        got = ours.encode(s)
        assert got == ref, (s, got, ref)
        assert ours.decode(got) == hf.decode(ref) == s


def test_bpe_synthetic_roundtrip_and_prompt_template():
    t = GPT2BPE(synthetic_words=False)
    assert t.synthetic
    prompt = "You are an intelligent assistant. Answer the following question in detail:\nQuestion: hi\nAnswer:"
    ids = t.encode(prompt)
    assert all(0 <= i < 256 for i in ids)
    assert t.decode(ids) == prompt
    # <|endoftext|> is special and skipped on decode; ids >= 256 decode to printable pseudo-words
    assert t.decode(ids + [50256]) == prompt
    assert t.decode([50256], skip_special_tokens=False) == "<|endoftext|>"
    assert t.encode("a<|endoftext|>b") == t.encode("a") + [50256] + t.encode("b")
    txt = t.decode([300, 4000, 50000])
    assert txt and txt.isprintable()


def test_bpe_synthetic_word_mode_lengths_and_roundtrip():
    t = GPT2BPE()
    assert t.synthetic and t.synthetic_words
    prompt = "You are an intelligent assistant. Answer the following question in detail:\nQuestion: hi\nAnswer:"
    ids = t.encode(prompt)
    assert 15 <= len(ids) <= 30  # real GPT-2 BPE: 23 tokens; byte level would be 93
    assert all(0 <= i < 50256 for i in ids)
    assert t.decode(ids) == prompt and t.encode(prompt) == ids
    # a small model vocabulary bounds the ids (gpt2-tiny: 1000 ids, EOS 999)
    tiny = GPT2BPE(eos_token_id=999)
    tids = tiny.encode(prompt + " and some more words to collide")
    assert max(tids) < 999 and tiny.decode(tids) == prompt + " and some more words to collide"


@pytest.fixture(scope="module")
def wp_vocab(tmp_path_factory):
    pytest.importorskip("tokenizers")
    from tokenizers import BertWordPieceTokenizer

    tok = BertWordPieceTokenizer(lowercase=True, strip_accents=True, clean_text=True)
    d = tmp_path_factory.mktemp("wp")
    corpus_file = d / "corpus.txt"
    corpus_file.write_text("\n".join(CORPUS))
    tok.train([str(corpus_file)], vocab_size=600, show_progress=False)
    tok.save_model(str(d))
    return tok, str(d / "vocab.txt")


def test_wordpiece_matches_hf_on_same_vocab(wp_vocab):
    hf, vocab = wp_vocab
    ours = BertWordPiece(vocab)
    for s in SAMPLES:
        if any(ord(c) > 0x2000 and not (0x4E00 <= ord(c) <= 0x9FFF) for c in s):
            continue  # non-Latin punctuation/emoji classes need full Unicode tables (no ICU here)
        ref = hf.encode(s).ids  # the trained tokenizer has no post-processor: no [CLS]/[SEP]
        got = ours.encode(s, max_length=0, add_special_tokens=False)
        assert got == ref, (s, got, ref)


def test_wordpiece_truncation_and_synthetic():
    t = BertWordPiece()
    ids = t.encode("word " * 1000)
    assert len(ids) == 512 and ids[0] == t.cls_token_id and ids[-1] == t.sep_token_id
    assert t.encode("Hello, World!") == t.encode("hello , world !")
    assert all(0 <= i < 30522 for i in t.encode("some random text 123"))
