"""Text tokenizer (csrc/tokenizer.cpp; web-rwkv Tokenizer as used at
src/dynamic_batch_manager.rs:512-515). Parity unpinned against web-rwkv itself (crate not
vendored); pinned by (1) the RWKV world vocabulary's own greedy longest-match encodings
(tests/golden/make_tokenizer_golden.py: TTS id = world id + 12292), (2) an
independent pure-Python pass over the TTS vocabulary JSON, (3) every vocabulary entry
round-tripping to its own id, (4) longest match winning on overlapping entries. CPU only."""
import json
import os

import pytest

from rwkvtts.tokenizer import Tokenizer, TokenizerError

HERE = os.path.dirname(os.path.abspath(__file__))
VOCAB = os.path.join(HERE, "..", "rwkv-tts-rs_amd", "assets", "tokenizer.json")


@pytest.fixture(scope="module")
def tok():
    return Tokenizer(VOCAB)


@pytest.fixture(scope="module")
def vocab():
    d = json.load(open(VOCAB, encoding="utf-8"))
    by_bytes = {}
    for k, v in d.items():
        b = v.encode("utf-8")
        by_bytes[b] = max(by_bytes.get(b, -1), int(k))
    return d, by_bytes


def test_golden_sentences(tok):
    g = json.load(open(os.path.join(HERE, "golden", "tokenizer_golden.json"), encoding="utf-8"))
    for c in g["cases"]:
        if c["tts_ids"] is None:
            with pytest.raises(TokenizerError):
                tok.encode(c["text"])
            continue
        ids = tok.encode(c["text"])
        assert ids == c["tts_ids"], c["text"]
        if c["world_whole_utf8"] and "<|" not in c["text"]:
            assert ids == c["world_plus_offset"], c["text"]   # the world vocab's own encoding
        assert tok.decode(ids) == c["text"].encode("utf-8")


def test_every_entry_roundtrips(tok, vocab):
    d, by_bytes = vocab
    assert tok.vocab_size == 77923
    for k, v in d.items():
        b = v.encode("utf-8")
        assert tok.encode(b) == [by_bytes[b]], (k, v)
        assert tok.decode([int(k)]) == b


def test_longest_match_wins(tok, vocab):
    d, by_bytes = vocab
    n = 0
    for b, i in sorted(by_bytes.items(), key=lambda x: -len(x[0])):
        if len(b) >= 4 and b[:-1] in by_bytes and b[:2] in by_bytes:
            assert tok.encode(b) == [i]                   # not prefix + rest
            assert tok.encode(b + b"!") == [i, by_bytes[b"!"]]
            n += 1
        if n > 200:
            break
    assert n > 50
    # special-token literals are vocabulary entries too (TAG_0 = 8193, spct_5 = 77828)
    assert tok.encode("<|tag_0|>") == [8193] and tok.encode("<|spct_5|>") == [77828]


def test_special_layout(tok):
    """world byte 'a' (world id 98) at 12390; EOS / tags / global / spct ranges."""
    assert tok.encode("a") == [98 + 12292]
    assert tok.decode([8192]) == b"<|semantic_token_eos|>"
    assert tok.decode([8196]) == b"<|global_token_0|>"
    assert tok.decode([77823]) == b"<|spct_0|>"


def test_errors(tok):
    with pytest.raises(TokenizerError):
        tok.encode("\U0001F600")  # needs raw byte tokens the TTS vocabulary cannot hold
    assert tok.encode("") == []
    with pytest.raises(Exception):
        Tokenizer('{"1": "a", "x": "b"}')
    t2 = Tokenizer('{"1": "ab", "2": "a", "3": "b", "4": [99, 100]}')
    assert t2.encode("abab") == [1, 1] and t2.encode("ba") == [3, 2] and t2.encode("cd") == [4]
