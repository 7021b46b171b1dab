"""Text tokenizer (host mirror of web-rwkv's `Tokenizer` as used by the reference:
src/shared_runtime.rs:187-192 builds it from assets/model/tokenizer.json, and
src/dynamic_batch_manager.rs:512-515 encodes the request text's UTF-8 bytes). Native code:
csrc/tokenizer.cpp (greedy longest match)."""
import ctypes
from typing import List, Sequence, Union

import numpy as np

from ._ffi import check, lib


class TokenizerError(ValueError):
    pass


class Tokenizer:
    def __init__(self, vocab: Union[str, bytes]):
        """vocab: the vocabulary JSON text (str / bytes), or a path to it."""
        if isinstance(vocab, str) and not vocab.lstrip().startswith("{"):
            with open(vocab, "rb") as f:
                vocab = f.read()
        if isinstance(vocab, str):
            vocab = vocab.encode("utf-8")
        h = ctypes.c_void_p()
        check(lib().rwkvtts_tokenizer_create(vocab, len(vocab), ctypes.byref(h)), "tokenizer_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().rwkvtts_tokenizer_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def vocab_size(self) -> int:
        return int(lib().rwkvtts_tokenizer_vocab_size(self._h))

    def encode(self, text: Union[str, bytes]) -> List[int]:
        b = text.encode("utf-8") if isinstance(text, str) else bytes(text)
        n = ctypes.c_size_t()
        out = np.zeros(max(len(b), 1), dtype=np.uint32)  # never more ids than bytes
        rc = lib().rwkvtts_tokenizer_encode(self._h, b, len(b), out.ctypes.data_as(ctypes.c_void_p), out.size,
                                            ctypes.byref(n))
        if rc != 0:
            raise TokenizerError(lib().rwkvtts_last_error().decode())
        return out[:n.value].tolist()

    def decode(self, ids: Sequence[int]) -> bytes:
        a = np.ascontiguousarray(np.asarray(ids, dtype=np.uint32))
        n = ctypes.c_size_t()
        check(lib().rwkvtts_tokenizer_decode(self._h, a.ctypes.data_as(ctypes.c_void_p), a.size, None, 0,
                                             ctypes.byref(n)), "tokenizer_decode")
        buf = ctypes.create_string_buffer(max(n.value, 1))
        check(lib().rwkvtts_tokenizer_decode(self._h, a.ctypes.data_as(ctypes.c_void_p), a.size, buf, n.value,
                                             ctypes.byref(n)), "tokenizer_decode")
        return buf.raw[:n.value]
