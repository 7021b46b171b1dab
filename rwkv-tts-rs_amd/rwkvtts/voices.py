"""RAF voice store: host mirror of `VoiceFeatureManager` (src/voice_feature_manager.rs:15-500).

A voice is `<raf_dir>/<id>.raf.json`, the `VoiceFeature` struct serialised by
`serde_json::to_vec_pretty` (field order as declared, 2-space indent, one array element per
line, UTF-8 text unescaped, f32 in shortest round-trip form, `created_at` as chrono's RFC 3339
with 0 / 3 / 6 / 9 fractional digits), whose `checksum` is the SHA-256 of the same
serialisation with `checksum: ""` (:169-235); loads verify it (:252-283). `voices_metadata.json`
holds `{"voices": [VoiceMetadata...]}` (to_string_pretty, :371-438). Ids are
`voice_%Y%m%d_%H%M%S_<8 hex of a v4 uuid>` (:153-158). The serialiser is pinned against the
reference's own RAF files (tests/golden/raf_full: recomputed checksums and bytes match).
"""
import datetime as _dt
import hashlib
import json
import os
import re
import threading
import uuid
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

_FEATURE_FIELDS = ("id", "name", "prompt_text", "created_at", "global_tokens", "semantic_tokens",
                   "audio_duration", "sample_rate", "checksum")
_META_FIELDS = ("id", "name", "prompt_text", "created_at", "file_path", "file_size", "checksum")


class F32:
    """An f32 value serialised the way serde_json (ryu) writes an f32: shortest round-trip."""

    def __init__(self, v):
        self.v = np.float32(v)

    def __float__(self):
        return float(self.v)

    def text(self) -> str:
        if not np.isfinite(self.v):
            return "null"
        s = np.format_float_positional(self.v, unique=True, trim="0")
        if "e" not in s and "." not in s:
            s += ".0"
        if s.endswith("."):
            s += "0"
        return s


def _pretty(v, ind: int = 0) -> str:
    """serde_json PrettyFormatter: '{' / '[' then one entry per line at +2, ': ' after keys."""
    pad, pad2 = "  " * ind, "  " * (ind + 1)
    if isinstance(v, dict):
        if not v:
            return "{}"
        items = [f"{pad2}{json.dumps(k, ensure_ascii=False)}: {_pretty(x, ind + 1)}" for k, x in v.items()]
        return "{\n" + ",\n".join(items) + "\n" + pad + "}"
    if isinstance(v, (list, tuple)):
        if not v:
            return "[]"
        return "[\n" + ",\n".join(pad2 + _pretty(x, ind + 1) for x in v) + "\n" + pad + "]"
    if isinstance(v, F32):
        return v.text()
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (int, np.integer)):
        return str(int(v))
    if v is None:
        return "null"
    return json.dumps(v, ensure_ascii=False)


def rfc3339_utc(t: _dt.datetime, nanos: Optional[int] = None) -> str:
    """chrono DateTime<Utc> serde form (SecondsFormat::AutoSi, 'Z')."""
    ns = t.microsecond * 1000 if nanos is None else nanos
    base = t.strftime("%Y-%m-%dT%H:%M:%S")
    if ns == 0:
        frac = ""
    elif ns % 1_000_000 == 0:
        frac = f".{ns // 1_000_000:03d}"
    elif ns % 1000 == 0:
        frac = f".{ns // 1000:06d}"
    else:
        frac = f".{ns:09d}"
    return base + frac + "Z"


@dataclass
class VoiceFeature:
    id: str
    name: str
    prompt_text: str
    created_at: str
    global_tokens: List[int]
    semantic_tokens: List[int]
    audio_duration: float
    sample_rate: int
    checksum: str = ""

    def serialise(self, checksum: Optional[str] = None) -> bytes:
        d = {k: getattr(self, k) for k in _FEATURE_FIELDS}
        d["audio_duration"] = F32(self.audio_duration)
        if checksum is not None:
            d["checksum"] = checksum
        return _pretty(d).encode("utf-8")

    def compute_checksum(self) -> str:
        return hashlib.sha256(self.serialise(checksum="")).hexdigest()


@dataclass
class VoiceMetadata:
    id: str
    name: str
    prompt_text: str
    created_at: str
    file_path: str
    file_size: int
    checksum: str


@dataclass
class CacheStats:
    total_voices: int = 0
    cache_hits: int = 0
    cache_misses: int = 0
    last_refresh: str = field(default_factory=lambda: rfc3339_utc(_dt.datetime.now(_dt.timezone.utc)))


class VoiceFeatureManager:
    def __init__(self, raf_dir: str):
        self.raf_dir = raf_dir
        self.metadata_file = os.path.join(raf_dir, "voices_metadata.json")
        os.makedirs(os.path.join(raf_dir, "temp", "upload_temp_files"), exist_ok=True)
        self._cache: Dict[str, VoiceFeature] = {}
        self._lock = threading.Lock()
        # serialises every metadata read-modify-write and RAF file write (concurrent extract /
        # delete / rename must not lose entries)
        self._io_lock = threading.RLock()
        self.stats = CacheStats()

    @classmethod
    def new_with_preload(cls, raf_dir: str) -> "VoiceFeatureManager":
        m = cls(raf_dir)
        m.preload_all_voices()
        return m

    def preload_all_voices(self) -> int:
        n = 0
        for meta in self.list_voices():
            try:
                self._load(meta.id, update_stats=False)
                n += 1
            except (OSError, ValueError):
                pass
        self.stats.total_voices = n
        return n

    @staticmethod
    def generate_voice_id(now: Optional[_dt.datetime] = None) -> str:
        now = now or _dt.datetime.now(_dt.timezone.utc)
        return f"voice_{now.strftime('%Y%m%d_%H%M%S')}_{str(uuid.uuid4())[:8]}"

    # Deliberate deviation from the reference (voice_feature_manager.rs:318 joins the id as given):
    # the id comes from unauthenticated request bodies, so anything that is not a plain file stem
    # ("../x", "/abs/x", "a/b") is refused instead of reading or deleting outside raf_dir.
    _ID_RE = re.compile(r"[A-Za-z0-9_\-]{1,128}")

    def _path(self, voice_id: str) -> str:
        if not isinstance(voice_id, str) or not self._ID_RE.fullmatch(voice_id):
            raise ValueError(f"invalid voice id: {voice_id!r}")
        return os.path.join(self.raf_dir, f"{voice_id}.raf.json")

    def save_voice_feature(self, name: str, prompt_text: str, global_tokens, semantic_tokens,
                           audio_duration: float, sample_rate: int) -> str:
        now = _dt.datetime.now(_dt.timezone.utc)
        vf = VoiceFeature(self.generate_voice_id(now), name, prompt_text, rfc3339_utc(now),
                          [int(x) for x in global_tokens], [int(x) for x in semantic_tokens],
                          float(np.float32(audio_duration)), int(sample_rate))
        vf.checksum = vf.compute_checksum()
        data = vf.serialise()
        path = self._path(vf.id)
        with self._io_lock:
            os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
            with open(path, "wb") as f:
                f.write(data)
            self._edit_metadata(lambda vs: vs + [VoiceMetadata(vf.id, name, prompt_text, vf.created_at, path,
                                                               len(data), vf.checksum)])
        with self._lock:
            self._cache[vf.id] = vf
        return vf.id

    def _load(self, voice_id: str, update_stats: bool) -> VoiceFeature:
        with self._lock:
            if voice_id in self._cache:
                if update_stats:
                    self.stats.cache_hits += 1
                return self._cache[voice_id]
            if update_stats:
                self.stats.cache_misses += 1
        path = self._path(voice_id)
        if not os.path.exists(path):
            raise FileNotFoundError(f"音色特征文件不存在: {voice_id}")
        with open(path, "rb") as f:
            d = json.loads(f.read().decode("utf-8"))
        vf = VoiceFeature(**{k: d[k] for k in _FEATURE_FIELDS})
        if vf.compute_checksum() != vf.checksum:
            raise ValueError(f"音色特征文件校验和不匹配: {voice_id}")
        with self._lock:
            self._cache[voice_id] = vf
        return vf

    def load_voice_feature(self, voice_id: str) -> VoiceFeature:
        return self._load(voice_id, update_stats=True)

    def get_voice_tokens(self, voice_id: str) -> Tuple[List[int], List[int]]:
        vf = self._load(voice_id, update_stats=True)
        return list(vf.global_tokens), list(vf.semantic_tokens)

    def list_voices(self) -> List[VoiceMetadata]:
        if not os.path.exists(self.metadata_file):
            return []
        with open(self.metadata_file, encoding="utf-8") as f:
            d = json.load(f)
        return [VoiceMetadata(**{k: v[k] for k in _META_FIELDS}) for v in d["voices"]]

    def _edit_metadata(self, fn):
        with self._io_lock:
            voices = fn(self.list_voices())
            text = _pretty({"voices": [{k: getattr(v, k) for k in _META_FIELDS} for v in voices]})
            os.makedirs(os.path.dirname(self.metadata_file) or ".", exist_ok=True)
            with open(self.metadata_file, "w", encoding="utf-8") as f:
                f.write(text)

    def delete_voice(self, voice_id: str) -> None:
        path = self._path(voice_id)
        with self._io_lock:
            if os.path.exists(path):
                os.remove(path)
            if os.path.exists(self.metadata_file):
                self._edit_metadata(lambda vs: [v for v in vs if v.id != voice_id])
        with self._lock:
            self._cache.pop(voice_id, None)

    def rename_voice(self, voice_id: str, new_name: str) -> None:
        vf = self.load_voice_feature(voice_id)
        vf = VoiceFeature(**{**vf.__dict__, "name": new_name})
        vf.checksum = vf.compute_checksum()
        with self._io_lock:
            with open(self._path(voice_id), "wb") as f:
                f.write(vf.serialise())
            if not os.path.exists(self.metadata_file):
                raise FileNotFoundError("元数据文件不存在")

            def upd(vs):
                for v in vs:
                    if v.id == voice_id:
                        v.name = new_name
                return vs
            self._edit_metadata(upd)
        with self._lock:
            self._cache[voice_id] = vf

    def clear_cache(self) -> None:
        with self._lock:
            self._cache.clear()
            self.stats = CacheStats()

    def refresh_cache(self) -> None:
        self.clear_cache()
        self.preload_all_voices()

    def get_cache_hit_rate(self) -> float:
        t = self.stats.cache_hits + self.stats.cache_misses
        return self.stats.cache_hits / t if t else 0.0

    def is_voice_cached(self, voice_id: str) -> bool:
        with self._lock:
            return voice_id in self._cache

    def get_cached_voice_count(self) -> int:
        with self._lock:
            return len(self._cache)
