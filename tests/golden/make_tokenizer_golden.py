"""Generates tests/golden/tokenizer_golden.json (run here, where /root/reference exists).

Independent pin for the text tokenizer (csrc/tokenizer.cpp): the RWKV "world" vocabulary that
the reference ships beside its Python assets (参考/python/rwkv_vocab_v20230424.txt: one
`id repr(token) length` line per token, str or bytes literal) is loaded with ast.literal_eval
(literals only, nothing executed) and a pure-Python greedy longest-match tokenizer encodes a set
of sentences. The TTS vocabulary (assets/model/tokenizer.json) places world id w at w + 12292
(SURVEY A.4), so where every matched world token is a whole UTF-8 string the TTS ids must be
world ids + 12292 (the TTS JSON cannot hold the world vocab's raw bytes 0x80-0xff: text that needs
them fails, see tokenizer.cpp). A second pure-Python pass over the TTS JSON itself gives the
expected ids for every sentence (None = NoMatchingTokenFound).
"""
import ast
import json
import os

REF = "/root/reference/参考/python/rwkv_vocab_v20230424.txt"
TTS = "/root/reference/assets/model/tokenizer.json"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tokenizer_golden.json")

SENTENCES = [
    "Hello world, this is a test of the RWKV text-to-speech tokenizer.",
    "The quick brown fox jumps over the lazy dog 1234567890!",
    "你好，世界！今天天气很好，我们一起去公园散步吧。",
    "RWKV-7 \"Goose\" uses a linear-time recurrent state; 32 global + 512 semantic tokens.",
    "Mixed 中英文 text with numbers 3.14159 and symbols @#$%^&*()_+-=[]{}|;':\",./<>?",
    "    leading spaces and\ttabs\nand newlines\r\n",
    "日本語のテキストも処理できます。한국어도 가능합니다.",
    "Über straße café naïve résumé — “quotes” and ‘single’ … ellipsis",
    "emoji are multi-byte: 😀🎉🚀",
    "<|tag_0|> is a literal in the TTS vocabulary but not in the world vocabulary",
]


def load_world(path):
    vocab = {}
    for ln in open(path, encoding="utf-8"):
        i = ln.index(" ")
        j = ln.rindex(" ")
        idx = int(ln[:i])
        tok = ast.literal_eval(ln[i + 1:j])
        b = tok.encode("utf-8") if isinstance(tok, str) else tok
        assert len(b) == int(ln[j + 1:])
        vocab[b] = idx
    return vocab


def _is_utf8(b):
    try:
        b.decode("utf-8")
        return True
    except UnicodeDecodeError:
        return False


def encode(vocab, maxlen, data):
    out, pos = [], 0
    while pos < len(data):
        for L in range(min(maxlen, len(data) - pos), 0, -1):
            t = vocab.get(data[pos:pos + L])
            if t is not None:
                out.append(t)
                pos += L
                break
        else:
            raise ValueError(f"no token at {pos}")
    return out


def load_tts(path):
    """The TTS vocabulary JSON itself (id -> string), byte strings -> highest id."""
    vocab = {}
    for k, v in json.load(open(path, encoding="utf-8")).items():
        b = v.encode("utf-8") if isinstance(v, str) else bytes(v)
        vocab[b] = max(vocab.get(b, -1), int(k))
    return vocab


def main():
    world = load_world(REF)
    wmax = max(len(b) for b in world)
    inv = {v: k for k, v in world.items()}
    tts = load_tts(TTS)
    tmax = max(len(b) for b in tts)
    cases = []
    for s in SENTENCES:
        data = s.encode("utf-8")
        ids = encode(world, wmax, data)
        whole = all(_is_utf8(inv[i]) for i in ids)  # no raw-byte tokens needed
        try:
            tts_ids = encode(tts, tmax, data)
        except ValueError:
            tts_ids = None  # NoMatchingTokenFound (raw bytes the TTS JSON cannot hold)
        cases.append({"text": s, "world_ids": ids, "world_whole_utf8": whole,
                      "world_plus_offset": [i + 12292 for i in ids], "tts_ids": tts_ids})
    json.dump({"source": "world ids: 参考/python/rwkv_vocab_v20230424.txt; tts ids: assets/model/tokenizer.json; "
                         "both by a pure-Python greedy longest match",
               "offset": 12292, "cases": cases}, open(OUT, "w"), ensure_ascii=False, indent=1)


if __name__ == "__main__":
    main()
