// tokenizer.cpp -- the text tokenizer of the reference's prompt path: web-rwkv 0.10.16
// `Tokenizer::new(&vocab_json)` / `Tokenizer::encode(bytes)` as called at
// src/shared_runtime.rs:187-192 and src/dynamic_batch_manager.rs:512-515 over
// assets/model/tokenizer.json (an object mapping decimal id -> token string; web-rwkv also
// accepts a byte array per token).
//
// Algorithm (web-rwkv's, restated; the crate is not vendored, so parity is pinned only by the
// vocabulary's own properties -- tests/test_tokenizer.py): at each byte position take the LONGEST
// vocabulary entry that matches the input bytes there, emit its id, advance past it; a position
// that no entry matches is an error (TokenizerError::NoMatchingTokenFound -> the request fails).
// Tokens are matched as the UTF-8 bytes of their JSON strings. Several byte strings appear
// under two ids in the shipped vocabulary (world-vocab byte tokens 0x80..0xff were stored as
// the code points U+0080..U+00FF, whose UTF-8 collides with the genuine 2-byte tokens); web-rwkv
// resolves such a collision by HashMap iteration order (not reproducible), this build by the
// highest id, i.e. the genuine multi-byte token.
#include <string.h>

#include <algorithm>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace rwkvtts {
namespace {

struct Tokenizer {
  std::unordered_map<std::string, uint32_t> to_id;
  std::vector<std::string> by_id;        // id -> bytes (empty for unused ids)
  std::vector<uint8_t> has_id;
  std::vector<std::vector<int>> lengths;  // first byte -> distinct token lengths, descending
};

// ---- a JSON reader for {"<id>": "<string>" | [bytes...], ...} --------------------------------
struct Json {
  const char* p;
  const char* e;
  std::string err;
  void ws() {
    while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }
  bool lit(char c) {
    ws();
    if (p < e && *p == c) {
      ++p;
      return true;
    }
    return false;
  }
  static void put_utf8(std::string& s, uint32_t cp) {
    if (cp < 0x80) {
      s += (char)cp;
    } else if (cp < 0x800) {
      s += (char)(0xC0 | (cp >> 6));
      s += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      s += (char)(0xE0 | (cp >> 12));
      s += (char)(0x80 | ((cp >> 6) & 0x3F));
      s += (char)(0x80 | (cp & 0x3F));
    } else {
      s += (char)(0xF0 | (cp >> 18));
      s += (char)(0x80 | ((cp >> 12) & 0x3F));
      s += (char)(0x80 | ((cp >> 6) & 0x3F));
      s += (char)(0x80 | (cp & 0x3F));
    }
  }
  bool hex4(uint32_t& v) {
    if (e - p < 4) return false;
    v = 0;
    for (int i = 0; i < 4; ++i) {
      const char c = *p++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
      else return false;
    }
    return true;
  }
  bool str(std::string& out) {
    out.clear();
    if (!lit('"')) return fail("expected a string");
    while (p < e && *p != '"') {
      if (*p != '\\') {
        out += *p++;
        continue;
      }
      if (++p >= e) return fail("bad escape");
      const char c = *p++;
      switch (c) {
        case '"': out += '"'; break;
        case '\\': out += '\\'; break;
        case '/': out += '/'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'n': out += '\n'; break;
        case 'r': out += '\r'; break;
        case 't': out += '\t'; break;
        case 'u': {
          uint32_t v;
          if (!hex4(v)) return fail("bad \\u escape");
          if (v >= 0xD800 && v < 0xDC00) {  // surrogate pair
            uint32_t lo;
            if (e - p < 6 || p[0] != '\\' || p[1] != 'u') return fail("lone surrogate");
            p += 2;
            if (!hex4(lo) || lo < 0xDC00 || lo >= 0xE000) return fail("bad surrogate pair");
            v = 0x10000 + ((v - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(out, v);
          break;
        }
        default: return fail("bad escape");
      }
    }
    if (p >= e) return fail("unterminated string");
    ++p;
    return true;
  }
  bool bytes(std::string& out) {  // [b0, b1, ...]
    out.clear();
    if (!lit('[')) return fail("expected [");
    if (lit(']')) return true;
    do {
      ws();
      long v = 0;
      int nd = 0;
      while (p < e && *p >= '0' && *p <= '9' && nd < 4) {
        v = v * 10 + (*p++ - '0');
        ++nd;
      }
      if (nd == 0 || v > 255) return fail("bad byte value");
      out += (char)v;
    } while (lit(','));
    if (!lit(']')) return fail("expected ]");
    return true;
  }
  bool fail(const char* m) {
    if (err.empty()) err = m;
    return false;
  }
};

int parse_vocab(const char* text, size_t n, Tokenizer& t, std::string& why) {
  Json j{text, text + n, {}};
  if (!j.lit('{')) {
    why = "vocabulary: expected a JSON object";
    return RWKVTTS_EINVAL;
  }
  std::string key, val;
  if (!j.lit('}')) {
    do {
      if (!j.str(key)) break;
      char* endp = nullptr;
      const unsigned long id = strtoul(key.c_str(), &endp, 10);
      if (key.empty() || *endp || id > 0xFFFFFFu) {
        j.fail("vocabulary key is not a token id");
        break;
      }
      if (!j.lit(':')) {
        j.fail("expected :");
        break;
      }
      j.ws();
      const bool ok = (j.p < j.e && *j.p == '[') ? j.bytes(val) : j.str(val);
      if (!ok) break;
      if (val.empty()) continue;  // an empty token can never be matched
      if (id >= t.by_id.size()) {
        t.by_id.resize(id + 1);
        t.has_id.resize(id + 1, 0);
      }
      t.by_id[id] = val;
      t.has_id[id] = 1;
      auto it = t.to_id.find(val);
      if (it == t.to_id.end() || it->second < id) t.to_id[val] = (uint32_t)id;
    } while (j.lit(','));
    if (j.err.empty() && !j.lit('}')) j.fail("expected }");
  }
  if (!j.err.empty()) {
    why = "vocabulary: " + j.err + " at byte " + std::to_string(j.p - text);
    return RWKVTTS_EINVAL;
  }
  t.lengths.assign(256, {});
  for (auto& kv : t.to_id) {
    auto& L = t.lengths[(uint8_t)kv.first[0]];
    const int len = (int)kv.first.size();
    bool seen = false;
    for (int x : L) seen |= x == len;
    if (!seen) L.push_back(len);
  }
  for (auto& L : t.lengths) std::sort(L.begin(), L.end(), [](int a, int b) { return a > b; });
  return RWKVTTS_OK;
}

}  // namespace
}  // namespace rwkvtts

using namespace rwkvtts;

struct rwkvtts_tokenizer {
  Tokenizer t;
};

extern "C" {

int rwkvtts_tokenizer_create(const char* vocab_json, size_t len, rwkvtts_tokenizer** out) {
  RT_CHECK(vocab_json && out, RWKVTTS_EINVAL, "tokenizer_create: null argument");
  *out = nullptr;
  rwkvtts_tokenizer* tk = new (std::nothrow) rwkvtts_tokenizer();
  RT_CHECK(tk, RWKVTTS_ENOMEM, "tokenizer_create: out of memory");
  std::string why;
  const int rc = parse_vocab(vocab_json, len, tk->t, why);
  if (rc != RWKVTTS_OK) {
    delete tk;
    set_error(why);
    return rc;
  }
  *out = tk;
  return RWKVTTS_OK;
}

int rwkvtts_tokenizer_destroy(rwkvtts_tokenizer* t) {
  delete t;
  return RWKVTTS_OK;
}

int rwkvtts_tokenizer_encode(const rwkvtts_tokenizer* tk, const uint8_t* text, size_t n, uint32_t* ids,
                             size_t cap, size_t* n_ids) {
  RT_CHECK(tk && n_ids && (n == 0 || text), RWKVTTS_EINVAL, "tokenizer_encode: null argument");
  const Tokenizer& t = tk->t;
  size_t pos = 0, k = 0;
  std::string probe;
  while (pos < n) {
    bool found = false;
    for (int len : t.lengths[text[pos]]) {
      if (pos + (size_t)len > n) continue;
      probe.assign((const char*)text + pos, (size_t)len);
      auto it = t.to_id.find(probe);
      if (it == t.to_id.end()) continue;
      if (k < cap && ids) ids[k] = it->second;
      ++k;
      pos += (size_t)len;
      found = true;
      break;
    }
    if (!found) {
      *n_ids = k;
      set_error("tokenizer: no matching token at byte " + std::to_string(pos));
      return RWKVTTS_EINVAL;
    }
  }
  *n_ids = k;
  RT_CHECK(k <= cap || !ids, RWKVTTS_EINVAL, "tokenizer_encode: output buffer too small");
  return RWKVTTS_OK;
}

int rwkvtts_tokenizer_decode(const rwkvtts_tokenizer* tk, const uint32_t* ids, size_t n, uint8_t* text, size_t cap,
                             size_t* n_bytes) {
  RT_CHECK(tk && n_bytes && (n == 0 || ids), RWKVTTS_EINVAL, "tokenizer_decode: null argument");
  const Tokenizer& t = tk->t;
  size_t k = 0;
  for (size_t i = 0; i < n; ++i) {
    RT_CHECK(ids[i] < t.by_id.size() && t.has_id[ids[i]], RWKVTTS_EINVAL, "tokenizer_decode: unknown id");
    const std::string& s = t.by_id[ids[i]];
    if (text && k + s.size() <= cap) memcpy(text + k, s.data(), s.size());
    k += s.size();
  }
  *n_bytes = k;
  RT_CHECK(k <= cap || !text, RWKVTTS_EINVAL, "tokenizer_decode: output buffer too small");
  return RWKVTTS_OK;
}

int64_t rwkvtts_tokenizer_vocab_size(const rwkvtts_tokenizer* tk) {
  return tk ? (int64_t)tk->t.by_id.size() : -1;
}

}  // extern "C"
