"""Server-layer mirror (bin/server.rs): WAV bytes, speed / pitch mapping, the /api/tts handler
and generate_speech's silence fallback, with a stand-in pipeline (CPU only); the GPU end-to-end
run is in tests/test_gpu_pipeline.py."""
import base64
import json
import os
import struct

import numpy as np
import pytest

from rwkvtts import server as SV
from rwkvtts.pipeline import LightweightTtsPipeline, LightweightTtsPipelineArgs

HERE = os.path.dirname(os.path.abspath(__file__))


def _expected_wav(pcm_i16):
    n = len(pcm_i16)
    h = b"RIFF" + struct.pack("<I", 36 + 2 * n) + b"WAVE" + b"fmt " + struct.pack("<IHHIIHH", 16, 1, 1, 16000, 32000, 2, 16)
    h += b"data" + struct.pack("<Q", 2 * n)  # server.rs:141: usize -> 8 bytes
    return h + struct.pack("<%dh" % n, *pcm_i16)


def test_wav_small_signal_is_scaled_up():
    # max 0.5 -> scale min(0.8 / 0.5, 10) = 1.6; x * 32767 truncated toward zero
    got = SV.convert_samples_to_wav([0.5, -0.25, 0.0, 0.1])
    assert got == _expected_wav([26213, -13106, 0, 5242])


def test_wav_loud_and_silent():
    assert SV.convert_samples_to_wav([2.0, -4.0, 1.0]) == _expected_wav([16383, -32767, 8191])
    assert SV.convert_samples_to_wav([0.0, 0.0]) == _expected_wav([0, 0])
    # tiny signal: scale capped at 10
    assert SV.convert_samples_to_wav([0.01, -0.02]) == _expected_wav([3276, -6553])


def test_speed_and_pitch_mapping():
    assert [SV.map_speed(x) for x in (None, "fast", "warp", 3.0, 3.4, 3.9, 4.2, 4.6, 4.8, 5.5, [1])] == [
        "medium", "fast", "medium", "very_slow", "very_slow", "slow", "medium", "fast", "fast", "very_fast", "medium"]
    assert SV.map_pitch("low_pitch") == "low" and SV.map_pitch(None) == "medium"
    # the remapped names miss PITCH_MAP -> pitch token 7 whatever was asked
    p = LightweightTtsPipeline.generate_property_tokens(LightweightTtsPipelineArgs(pitch=SV.map_pitch("high_pitch")))
    assert p[4] == 77823 + 7


class FakeManager:
    def __init__(self, result=([1] * 32, [5, 6, 7])):
        self.result = result
        self.seen = []

    def _tokens(self, text):
        if "\U0001F600" in text:
            raise ValueError("no matching token")
        return [ord(c) % 100 + 12293 for c in text]

    def generate_tts_batch(self, reqs):
        self.seen.extend(reqs)
        return [self.result for _ in reqs]


class FakeCodec:
    def decode_audio(self, g, s):
        return np.full(len(s) * 320, 0.25, dtype=np.float32)

    def decode_audio_batch(self, items):
        return [np.full(len(s) * 320, 0.25, dtype=np.float32) if s else np.zeros(0, np.float32) for _, s in items]


def test_handler_normal_and_zero_shot(tmp_path):
    m = FakeManager()
    pipe = LightweightTtsPipeline(m, FakeCodec())
    code, body = SV.handle_tts_json(json.dumps({"text": "hi", "speed": 4.6, "pitch": "high_pitch", "seed": 3}), pipe,
                                    str(tmp_path))
    assert code == 200 and body["success"] and body["rtf"] >= 0
    wav = base64.b64decode(body["audio_base64"])
    assert wav == SV.convert_samples_to_wav(np.full(3 * 320, 0.25, np.float32))
    req = m.seen[-1]
    assert req.property_tokens == [77823, 77823 + 15, 77823 + 47, 77823 + 22, 77823 + 7, 77823 + 4]  # male default
    assert req.args.seed == 3 and req.args.top_k == 100 and req.args.max_tokens == 8000
    # zero-shot by voice_id: RAF tokens passed, no property tokens
    raf = json.load(open(os.path.join(HERE, "golden", "raf_voice_05d8f5ed.json")))
    vid = SV.voice_manager(str(tmp_path)).save_voice_feature("v1", "x", raf["global_tokens"],
                                                              raf["semantic_tokens"][:9], 1.5, 16000)
    code, body = SV.handle_tts_json({"text": "hi", "voice_id": vid}, pipe, str(tmp_path))
    assert code == 200
    req = m.seen[-1]
    assert req.property_tokens == [] and req.ref_global_tokens == raf["global_tokens"]
    code, body = SV.handle_tts_json({"text": "hi", "voice_id": "nope"}, pipe, str(tmp_path))
    assert code == 400 and not body["success"]
    assert SV.handle_tts_json(b"{not json", pipe)[0] == 400


def test_generate_speech_silence_fallback():
    """A failed request (empty result) becomes 16000 zeros (lightweight_tts_pipeline.rs:828-830);
    untokenisable text fails its request the same way."""
    pipe = LightweightTtsPipeline(FakeManager(result=([], [])), FakeCodec())
    out = pipe.generate_speech(LightweightTtsPipelineArgs(text="abc"))
    assert out.shape == (16000,) and not out.any()
    pipe2 = LightweightTtsPipeline(FakeManager(), FakeCodec())
    out2 = pipe2.generate_speech(LightweightTtsPipelineArgs(text="bad \U0001F600"))
    assert out2.shape == (16000,) and not out2.any()
    outs = pipe2.generate_speech_batch([LightweightTtsPipelineArgs(text="ok"), LightweightTtsPipelineArgs(text="\U0001F600")])
    assert outs[0].size == 3 * 320 and outs[1].size == 0


def test_fastapi_route():
    pytest.importorskip("fastapi")
    from fastapi.testclient import TestClient
    app = SV.create_app(LightweightTtsPipeline(FakeManager(), FakeCodec()))
    r = TestClient(app).post("/api/tts", json={"text": "hello"})
    assert r.status_code == 200 and r.json()["success"]


def test_fastapi_voice_routes(tmp_path):
    pytest.importorskip("fastapi")
    from fastapi.testclient import TestClient

    class Pipe(LightweightTtsPipeline):
        @staticmethod
        def reference_tokenizer(path):
            return list(range(32)), [1, 2]
    c = TestClient(SV.create_app(Pipe(FakeManager(), FakeCodec()), voice_dir=str(tmp_path)))
    assert c.get("/api/voice-clone/list").json() == {"success": True, "voices": []}
    assert c.post("/api/voice-clone/extract", data={"voice_name": "n"}).json()["message"] == "需要上传音频文件"
    try:  # multipart parsing needs python-multipart (not installed in every image)
        import multipart  # noqa: F401
        have_mp = True
    except ImportError:
        have_mp = False
    if have_mp:
        import io
        import wave
        buf = io.BytesIO()
        with wave.open(buf, "wb") as w:
            w.setnchannels(1)
            w.setsampwidth(2)
            w.setframerate(16000)
            w.writeframes(b"\x10\x00" * 3200)
        r = c.post("/api/voice-clone/extract", data={"voice_name": "n", "prompt_text": "p"},
                   files={"audio_file": ("ref.wav", buf.getvalue(), "audio/wav")}).json()
        assert r["success"], r
        vid = r["voice_id"]
        assert not os.listdir(tmp_path / "temp" / "upload_temp_files")  # upload temp removed
    else:
        vid = SV.voice_manager(str(tmp_path)).save_voice_feature("n", "p", list(range(32)), [1, 2], 0.2, 16000)
    assert [v["id"] for v in c.get("/api/voice-clone/list").json()["voices"]] == [vid]
    assert c.post("/api/voice-clone/delete", json={"voice_id": vid}).json()["success"]
    assert c.get("/api/voice-clone/list").json()["voices"] == []
