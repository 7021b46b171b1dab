"""RAF voice store (rwkvtts/voices.py, src/voice_feature_manager.rs) and the voice-clone routes
(bin/server.rs:777-979): serialisation pinned byte-for-byte against the reference's own RAF
files, checksum verification, save / list / rename / delete, route bodies."""
import json
import os
import re
import shutil
import struct
import wave

import numpy as np
import pytest

from rwkvtts import server as SV
from rwkvtts.voices import VoiceFeature, VoiceFeatureManager, _FEATURE_FIELDS, _pretty

HERE = os.path.dirname(os.path.abspath(__file__))
RAF = os.path.join(HERE, "golden", "raf_full")
IDS = ["voice_20251014_130750_05d8f5ed", "voice_20251014_132429_d897f5e1"]


@pytest.mark.parametrize("vid", IDS)
def test_reference_raf_bytes_and_checksum(vid):
    raw = open(os.path.join(RAF, f"{vid}.raf.json"), "rb").read()
    d = json.loads(raw.decode("utf-8"))
    vf = VoiceFeature(**{k: d[k] for k in _FEATURE_FIELDS})
    assert vf.serialise() == raw                  # serde_json::to_vec_pretty, byte for byte
    assert vf.compute_checksum() == d["checksum"]  # SHA-256 with checksum ""
    meta = open(os.path.join(RAF, "voices_metadata.json"), "rb").read()
    assert _pretty(json.loads(meta.decode("utf-8"))).encode("utf-8") == meta


def test_store_loads_reference_files(tmp_path):
    for f in os.listdir(RAF):
        shutil.copy(os.path.join(RAF, f), tmp_path / f)
    m = VoiceFeatureManager.new_with_preload(str(tmp_path))
    assert m.get_cached_voice_count() == 2
    assert [v.id for v in m.list_voices()] == IDS
    g, s = m.get_voice_tokens(IDS[0])
    assert len(g) == 32 and s[:3] == [6652, 6858, 3037]
    assert m.stats.cache_hits == 1 and m.get_cache_hit_rate() == 1.0
    # a tampered file fails its checksum (after the cache is dropped)
    p = tmp_path / f"{IDS[1]}.raf.json"
    p.write_bytes(p.read_bytes().replace(b'"sample_rate": 24000', b'"sample_rate": 24001'))
    m.clear_cache()
    with pytest.raises(ValueError):
        m.load_voice_feature(IDS[1])


def test_save_rename_delete(tmp_path):
    m = VoiceFeatureManager(str(tmp_path))
    assert (tmp_path / "temp" / "upload_temp_files").is_dir()
    vid = m.save_voice_feature("名字", "提示", [1, 2, 3], [4, 5], 2.5, 16000)
    assert re.fullmatch(r"voice_\d{8}_\d{6}_[0-9a-f]{8}", vid)
    m2 = VoiceFeatureManager(str(tmp_path))  # fresh cache: read back from disk, checksum verified
    vf = m2.load_voice_feature(vid)
    assert (vf.name, vf.global_tokens, vf.semantic_tokens, vf.sample_rate) == ("名字", [1, 2, 3], [4, 5], 16000)
    assert m2.list_voices()[0].file_size == os.path.getsize(tmp_path / f"{vid}.raf.json")
    m2.rename_voice(vid, "新名字")
    assert VoiceFeatureManager(str(tmp_path)).load_voice_feature(vid).name == "新名字"
    assert m2.list_voices()[0].name == "新名字"
    m2.delete_voice(vid)
    assert m2.list_voices() == [] and not (tmp_path / f"{vid}.raf.json").exists()


def _wav(path, n=1600, sr=16000):
    with wave.open(str(path), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(sr)
        w.writeframes(struct.pack(f"<{n}h", *([1000] * n)))


def test_voice_routes(tmp_path):
    d = str(tmp_path)
    assert SV.handle_voice_list(d) == (200, {"success": True, "voices": []})
    assert SV.handle_voice_extract({}, None, None, d, is_multipart=False)[1]["message"] == "需要上传音频文件"
    assert SV.handle_voice_extract({"prompt_text": "p"}, None, None, d)[1]["message"] == "音色名称不能为空"
    assert SV.handle_voice_extract({"voice_name": "n"}, None, None, d)[1]["message"] == "提示词不能为空"
    assert SV.handle_voice_extract({"voice_name": "n", "prompt_text": "p"}, None, None, d)[1]["message"] == "未找到音频文件"
    wav = tmp_path / "a.wav"
    _wav(wav)
    # no BiCodecTokenize encoder: the reference's extraction-failure body
    code, body = SV.handle_voice_extract({"voice_name": "n", "prompt_text": "p"}, str(wav), None, d)
    assert not body["success"] and body["message"].startswith("音频特征提取失败") and body["voice_id"] is None

    class Pipe:
        @staticmethod
        def reference_tokenizer(path):
            return list(range(32)), [7, 8, 9]
    code, body = SV.handle_voice_extract({"voice_name": "n", "prompt_text": "p"}, str(wav), Pipe(), d)
    assert body["success"] and body["message"] == "音色特征提取成功"
    vid = body["voice_id"]
    vf = SV.voice_manager(d).load_voice_feature(vid)
    assert vf.global_tokens == list(range(32)) and abs(vf.audio_duration - 0.1) < 1e-6 and vf.sample_rate == 16000
    code, body = SV.handle_voice_list(d)
    assert body["success"] and [v["id"] for v in body["voices"]] == [vid]
    assert SV.handle_voice_delete(b"{bad", d)[1] == {"success": False, "message": "请求格式错误"}
    assert SV.handle_voice_delete(json.dumps({"voice_id": vid}), d)[1] == {"success": True, "message": "音色删除成功"}
    assert SV.handle_voice_list(d)[1]["voices"] == []


def test_voice_id_path_traversal_refused(tmp_path):
    """Deliberate deviation from voice_feature_manager.rs:318: ids from request bodies that are not
    a plain file stem never reach the filesystem (no read / delete outside raf_dir)."""
    import pytest
    from rwkvtts.voices import VoiceFeatureManager
    outside = tmp_path / "victim.raf.json"
    outside.write_text("{}")
    m = VoiceFeatureManager(str(tmp_path / "raf"))
    for bad in ("../victim", str(tmp_path / "victim"), "a/b", "..", "", "x\x00y"):
        with pytest.raises(ValueError):
            m.delete_voice(bad)
        with pytest.raises(ValueError):
            m.load_voice_feature(bad)
    assert outside.exists()


def test_concurrent_saves_keep_every_entry(tmp_path):
    import threading
    from rwkvtts.voices import VoiceFeatureManager
    m = VoiceFeatureManager(str(tmp_path / "raf"))
    ids = []
    ths = [threading.Thread(target=lambda i=i: ids.append(m.save_voice_feature(f"v{i}", "t", [1] * 32, [2] * 4, 1.0, 16000)))
           for i in range(12)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert sorted(v.id for v in m.list_voices()) == sorted(ids) and len(set(ids)) == 12
