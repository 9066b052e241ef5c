"""Tokenizer parity with HuggingFace (VERDICT r5 'missing' #2): the native pipeline
``torch.ops.pcmp.text_encode`` (csrc/runtime/text_core.h) and its pure-Python twin
(``data.imdb.encode(force_python=True)``) against ``transformers.BertTokenizer(vocab,
do_lower_case=True).encode(text, add_special_tokens=True, max_length=128, truncation=True)`` post-padded
to 128 -- the reference's tokenisation (/root/reference/pytorch_on_language_distr.py:56-81) -- on
HTML-stripped reviews with accents, combining marks, CJK, Hangul, Unicode punctuation / whitespace /
format characters, fullwidth forms, emoji, over-long words and truncation.  The vocabulary is built
offline from HuggingFace's OWN normaliser + pre-tokeniser output (no download), kept small so that
WordPiece continuations and [UNK] are exercised.
"""
import collections

import pytest
import torch

from pcmp.data import imdb

transformers = pytest.importorskip("transformers")

REVIEWS = [
    "One of the other reviewers has mentioned that after watching just 1 Oz episode you'll be hooked.<br /><br />"
    "They are right, as this is exactly what happened with me.",
    "A wonderful little production. <br /><br />The filming technique is very unassuming- very old-time-BBC fashion.",
    "Café society: the naïve résumé of Zoë at the Ångström Hôtel — “brilliant”, ‘superb’… ¡Olé! ¿Qué?",
    "Combining marks: école, ño, Å; Greek ΑΘΗΝΑ and Cyrillic ПРИВЕТ МИР!",
    "中国电影很好看。日本の映画も良い！ 한국 영화 안녕하세요 — 最高",
    "Fullwidth ＡＢＣ１２３ and ligature ﬁne, emoji 😀👍 and symbols © ® ™ ° ± ×.",
    "Zero​width‍spaces, NBSP here, ideographic　space, tab\tand\nnewline\r\nend.",
    "Supercalifragilisticexpialidocious" * 4 + " is over a hundred characters; "
    "pneumonoultramicroscopicsilicovolcanoconiosis is not.",
    "Numbers 1,234.56 and $7.89 (twenty-three%) [brackets] {braces} <notatag and a > b",
    " ".join(["word"] * 200) + " truncated tail that never appears",
    "Mixed CASE WoRdS, URLs http://example.com/path?x=1&y=2 and e-mails name@site.org!!!",
    "Accented capitals ÉÈÊË ÀÂÄ ÎÏ ÔÖ ÙÛÜ Ç Ñ ß ẞ Ø Æ Œ Ł Đ Ħ — dashes –‐‒ and quotes «» „“",
    "",
    "<i>only tags</i><b></b>",
]


def _hf_tokenize_words(tok, text):
    bt = tok.backend_tokenizer
    norm = bt.normalizer.normalize_str(text)
    return [w for w, _ in bt.pre_tokenizer.pre_tokenize_str(norm)]


@pytest.fixture(scope="module")
def vocab_and_hf(tmp_path_factory):
    d = tmp_path_factory.mktemp("vocab")
    # bootstrap a tokenizer with specials only, to run HuggingFace's normaliser / pre-tokeniser
    specials = ["[PAD]"] + [f"[unused{i}]" for i in range(99)] + ["[UNK]", "[CLS]", "[SEP]", "[MASK]"]
    boot = d / "boot.txt"
    boot.write_text("\n".join(specials) + "\n", encoding="utf-8")
    hf0 = transformers.BertTokenizer(vocab=str(boot), do_lower_case=True)
    texts = [imdb.rm_tags(t) for t in REVIEWS]
    cnt = collections.Counter()
    chars = set()
    for t in texts:
        for w in _hf_tokenize_words(hf0, t):
            cnt[w] += 1
            chars.update(w)
    vocab = list(specials)
    seen = set(vocab)
    # single characters and their continuations (most of them), then the frequent whole words and a
    # few word pieces: WordPiece then splits the rest, and a few characters stay [UNK]
    drop = {"😀", "ß"}
    for c in sorted(chars):
        for p in (c, "##" + c):
            if c not in drop and p not in seen:
                vocab.append(p); seen.add(p)
    for w, _ in cnt.most_common(60):
        if w not in seen:
            vocab.append(w); seen.add(w)
    for p in ("##ing", "##ed", "##er", "##tion", "##ly", "super", "##cal", "film", "##s"):
        if p not in seen:
            vocab.append(p); seen.add(p)
    path = d / "vocab.txt"
    path.write_text("\n".join(vocab) + "\n", encoding="utf-8")
    hf = transformers.BertTokenizer(vocab=str(path), do_lower_case=True)
    return vocab, hf


def _hf_ids(hf, texts, max_len=128):
    out = torch.zeros(len(texts), max_len, dtype=torch.long)
    for n, t in enumerate(texts):
        ids = hf.encode(imdb.rm_tags(t), add_special_tokens=True, max_length=max_len, truncation=True)
        out[n, :len(ids)] = torch.tensor(ids)
    return out


def test_native_encode_matches_huggingface(vocab_and_hf):
    from pcmp.ops import _lib
    if not (_lib.load() and hasattr(torch.ops.pcmp, "text_encode")):
        pytest.skip(f"native library not built: {_lib.load_error()}")
    vocab, hf = vocab_and_hf
    ref = _hf_ids(hf, REVIEWS)
    ids, mask = imdb.encode(REVIEWS, vocab, 128)
    for n in range(len(REVIEWS)):
        assert torch.equal(ids[n], ref[n]), (n, REVIEWS[n][:60], hf.convert_ids_to_tokens(ref[n][ref[n] > 0].tolist()),
                                              [vocab[i] for i in ids[n][ids[n] > 0].tolist()])
    assert torch.equal(mask, (ref > 0).long())
    assert (ids == 100).any() and (ids > 103).any()   # [UNK] and real pieces both exercised


def test_python_fallback_matches_huggingface(vocab_and_hf):
    vocab, hf = vocab_and_hf
    ref = _hf_ids(hf, REVIEWS)
    ids, mask = imdb.encode(REVIEWS, vocab, 128, force_python=True)
    for n in range(len(REVIEWS)):
        assert torch.equal(ids[n], ref[n]), (n, REVIEWS[n][:60])
    assert torch.equal(mask, (ref > 0).long())


def test_short_max_len_truncation(vocab_and_hf):
    from pcmp.ops import _lib
    if not _lib.load():
        pytest.skip("native library not built")
    vocab, hf = vocab_and_hf
    ref = _hf_ids(hf, REVIEWS, max_len=16)
    ids, _ = imdb.encode(REVIEWS, vocab, 16)
    assert torch.equal(ids, ref)
