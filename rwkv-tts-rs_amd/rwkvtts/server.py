"""The reference's HTTP API surface for the TTS path (bin/server.rs), over LightweightTtsPipeline.

* `convert_samples_to_wav` (:98-148): peak rule (max|x| > 1 -> 1/max, else min(0.8/max, 10),
  silence -> 1), f32 arithmetic, clamp to [-1, 1], x 32767 truncated to i16, 16 kHz mono WAV.
  The reference writes the data-chunk size as a usize (8 little-endian bytes on 64-bit) and
  declares RIFF size 36 + 2n; both are reproduced so the bytes match.
* `calculate_rtf` (:151-159), the speed / pitch string mapping of `handle_tts_json` (:528-584,
  including SURVEY B4: the pitch is remapped to names PITCH_MAP does not contain, so the pitch
  token is always 7), the voice lookup by voice_id (:481-515, a RAF JSON under `voice_dir`).
* `handle_tts_json(body, pipeline, voice_dir)` returns (HTTP status, JSON dict) exactly as the
  handler renders them; `create_app` wires it to POST /api/tts with FastAPI when installed.
* The voice-clone routes (:777-979, routes :1448-1450) over the RAF store (`voices.py`,
  VoiceFeatureManager): `handle_voice_list`, `handle_voice_delete`, `handle_voice_extract`
  (multipart voice_name / prompt_text / audio_file; the feature extraction needs the
  BiCodecTokenize + wav2vec2 encoders, whose graphs are absent: a pipeline may supply
  `reference_tokenizer`, otherwise the route answers the reference's extraction-failure body).
The embedded web UI and model download are out of scope.
"""
import base64
import json
import os
import time
from typing import Optional, Tuple

import numpy as np

from .pipeline import LightweightTtsPipelineArgs


def convert_samples_to_wav(samples, sample_rate: int = 16000) -> bytes:
    x = np.asarray(samples, dtype=np.float32)
    max_abs = np.float32(np.max(np.abs(x))) if x.size else np.float32(0.0)
    if max_abs > 0.0:
        scale = np.float32(1.0) / max_abs if max_abs > 1.0 else min(np.float32(0.8) / max_abs, np.float32(10.0))
    else:
        scale = np.float32(1.0)
    scale = np.float32(scale)
    y = np.clip(x * scale, np.float32(-1.0), np.float32(1.0)) * np.float32(32767.0)
    pcm = np.trunc(y).astype("<i2")  # Rust `as i16`: truncation toward zero
    n = x.size
    hdr = b"RIFF" + int(36 + n * 2).to_bytes(4, "little", signed=False) + b"WAVE"
    hdr += b"fmt " + (16).to_bytes(4, "little") + (1).to_bytes(2, "little") + (1).to_bytes(2, "little")
    hdr += int(sample_rate).to_bytes(4, "little") + int(sample_rate * 2).to_bytes(4, "little")
    hdr += (2).to_bytes(2, "little") + (16).to_bytes(2, "little")
    hdr += b"data" + int(n * 2).to_bytes(8, "little")  # (samples.len() * 2).to_le_bytes(): usize
    return hdr + pcm.tobytes()


def calculate_rtf(audio, processing_seconds: float) -> float:
    dur = len(audio) / 16000.0
    return processing_seconds / dur if dur > 0 else 0.0


def map_speed(speed) -> str:
    """:528-554: a known speed string passes through, other strings -> medium; numbers are
    bucketed (<=3.4 very_slow, <=4.0 slow, <=4.5 medium, <=4.8 fast, else very_fast); absent or
    unparsable -> medium (a non-number non-string parses as 4.2 -> medium)."""
    if speed is None:
        return "medium"
    if isinstance(speed, str):
        return speed if speed in ("very_slow", "slow", "medium", "fast", "very_fast") else "medium"
    try:
        v = float(np.float32(speed)) if isinstance(speed, (int, float)) and not isinstance(speed, bool) else 4.2
    except (TypeError, ValueError):
        v = 4.2
    if v <= float(np.float32(3.4)):
        return "very_slow"
    if v <= 4.0:
        return "slow"
    if v <= 4.5:
        return "medium"
    if v <= float(np.float32(4.8)):
        return "fast"
    return "very_fast"


def map_pitch(pitch: Optional[str]) -> str:
    """:570-576 (these names miss PITCH_MAP, so the pitch token is always 7)."""
    return {"low_pitch": "low", "medium_pitch": "medium", "high_pitch": "high",
            "very_high_pitch": "very_high"}.get(pitch, "medium")


_MANAGERS = {}


def voice_manager(voice_dir: str):
    """One VoiceFeatureManager per RAF directory (the server's AppState.voice_manager)."""
    from .voices import VoiceFeatureManager
    m = _MANAGERS.get(voice_dir)
    if m is None:
        m = _MANAGERS[voice_dir] = VoiceFeatureManager(voice_dir)
    return m


def load_voice_feature(voice_dir: str, voice_id: str) -> dict:
    """VoiceFeatureManager::load_voice_feature (checksum verified, cached)."""
    vf = voice_manager(voice_dir).load_voice_feature(voice_id)
    return dict(vf.__dict__)


def handle_tts_json(body, pipeline, voice_dir: str = "assets/raf") -> Tuple[int, dict]:
    t0 = time.perf_counter()
    if isinstance(body, (bytes, str)):
        try:
            body = json.loads(body)
        except ValueError as e:
            return 400, {"success": False, "error": f"JSON解析失败: {e}"}
    if not isinstance(body, dict) or not isinstance(body.get("text"), str):
        return 400, {"success": False, "error": "JSON解析失败: missing field `text`"}
    voice_id = body.get("voice_id")
    voice = None
    prompt_from_voice = None
    if voice_id:  # a non-empty voice_id loads the stored voice feature
        try:
            voice = load_voice_feature(voice_dir, voice_id)
            prompt_from_voice = voice.get("prompt_text", "")
        except (OSError, ValueError) as e:
            return 400, {"success": False, "error": f"音色ID '{voice_id}' 不存在或加载失败: {e}"}
    prompt_text = prompt_from_voice if prompt_from_voice is not None else (body.get("prompt_text") or "")
    args = LightweightTtsPipelineArgs(
        text=body["text"], ref_audio_path="", zero_shot=voice_id is not None,
        temperature=float(body.get("temperature") if body.get("temperature") is not None else 1.0),
        top_p=float(body.get("top_p") if body.get("top_p") is not None else 0.90),
        top_k=100, max_tokens=8000, seed=body.get("seed"),
        age=body.get("age") or "youth-adult", gender=body.get("gender") or "male",
        emotion=body.get("emotion") or "NEUTRAL", pitch=map_pitch(body.get("pitch")),
        speed=map_speed(body.get("speed")), prompt_text=prompt_text,
        voice_global_tokens=list(voice["global_tokens"]) if voice else None,
        voice_semantic_tokens=list(voice["semantic_tokens"]) if voice else None)
    try:
        audio = pipeline.generate_speech(args)
    except Exception as e:  # noqa: BLE001 -- rendered as the reference's 500 body
        return 500, {"success": False, "error": f"生成TTS音频失败: {e}"}
    wav = convert_samples_to_wav(audio, 16000)
    b64 = base64.standard_b64encode(wav).decode("ascii")
    total = time.perf_counter() - t0
    return 200, {"success": True, "message": "TTS生成成功", "audio_base64": b64,
                 "duration_ms": int(total * 1000), "rtf": calculate_rtf(audio, total)}


def handle_voice_list(voice_dir: str = "assets/raf") -> Tuple[int, dict]:
    """:920-944: {success, voices: [VoiceMetadata]} (an unreadable store: success false, [])."""
    try:
        voices = voice_manager(voice_dir).list_voices()
        return 200, {"success": True, "voices": [dict(v.__dict__) for v in voices]}
    except (OSError, ValueError, KeyError):
        return 200, {"success": False, "voices": []}


def handle_voice_delete(body, voice_dir: str = "assets/raf") -> Tuple[int, dict]:
    """:946-979: JSON {voice_id} -> {success, message}."""
    try:
        if isinstance(body, (bytes, str)):
            body = json.loads(body)
        voice_id = body["voice_id"]
        if not isinstance(voice_id, str):
            raise TypeError
    except (ValueError, KeyError, TypeError):
        return 200, {"success": False, "message": "请求格式错误"}
    try:
        voice_manager(voice_dir).delete_voice(voice_id)
        return 200, {"success": True, "message": "音色删除成功"}
    except (OSError, ValueError) as e:
        return 200, {"success": False, "message": f"删除音色失败: {e}"}


def handle_voice_extract(form: Optional[dict], audio_path: Optional[str], pipeline=None,
                         voice_dir: str = "assets/raf", is_multipart: bool = True) -> Tuple[int, dict]:
    """:777-918. form: voice_name / prompt_text; audio_path: the uploaded audio_file saved to a
    temporary path (None: no file). Extraction = pipeline.reference_tokenizer(path) ->
    (global, semantic) (the BiCodecTokenize encoders), duration / rate from the WAV itself."""
    def fail(msg):
        return 200, {"success": False, "message": msg, "voice_id": None}
    if not is_multipart:
        return fail("需要上传音频文件")
    form = form or {}
    name, prompt = form.get("voice_name") or "", form.get("prompt_text") or ""
    if not name:
        return fail("音色名称不能为空")
    if not prompt:
        return fail("提示词不能为空")
    if not audio_path:
        return fail("未找到音频文件")
    try:
        tok = getattr(pipeline, "reference_tokenizer", None)
        if tok is None:
            raise RuntimeError("ONNX模型文件不存在: assets/model/BiCodecTokenize.onnx")
        g, sem = tok(audio_path)
        from .audio import read_wav
        x, sr, ch = read_wav(audio_path)
        duration = (x.size // max(ch, 1)) / float(sr)
    except Exception as e:  # noqa: BLE001 -- the reference renders every extraction error this way
        return fail(f"音频特征提取失败: {e}")
    try:
        vid = voice_manager(voice_dir).save_voice_feature(name, prompt, list(g), list(sem), duration, sr)
    except (OSError, ValueError) as e:
        return fail(f"音色特征提取失败: {e}")
    return 200, {"success": True, "message": "音色特征提取成功", "voice_id": vid}


def create_app(pipeline, voice_dir: str = "assets/raf"):
    """FastAPI app with POST /api/tts (server.rs:1447). Serve with uvicorn."""
    from fastapi import FastAPI, Request
    from fastapi.responses import JSONResponse

    app = FastAPI(title="rwkvtts (MI355X)")

    @app.post("/api/tts")
    async def api_tts(request: Request):
        import anyio
        body = await request.body()
        code, payload = await anyio.to_thread.run_sync(handle_tts_json, body, pipeline, voice_dir)
        return JSONResponse(payload, status_code=code)

    @app.get("/api/voice-clone/list")
    async def api_voice_list():
        code, payload = handle_voice_list(voice_dir)
        return JSONResponse(payload, status_code=code)

    @app.post("/api/voice-clone/delete")
    async def api_voice_delete(request: Request):
        code, payload = handle_voice_delete(await request.body(), voice_dir)
        return JSONResponse(payload, status_code=code)

    @app.post("/api/voice-clone/extract")
    async def api_voice_extract(request: Request):
        import anyio
        import tempfile
        ctype = request.headers.get("content-type", "")
        if not ctype.startswith("multipart/"):
            return JSONResponse(handle_voice_extract(None, None, pipeline, voice_dir, is_multipart=False)[1])
        form = await request.form()
        fields = {k: v for k, v in form.items() if isinstance(v, str)}
        up = form.get("audio_file")
        path = None
        if up is not None and not isinstance(up, str):
            ext = os.path.splitext(up.filename or "audio")[1] or ".wav"
            tmp_dir = os.path.join(voice_dir, "temp", "upload_temp_files")
            os.makedirs(tmp_dir, exist_ok=True)
            fd, path = tempfile.mkstemp(suffix=ext, dir=tmp_dir)
            with os.fdopen(fd, "wb") as f:
                f.write(await up.read())
        try:
            code, payload = await anyio.to_thread.run_sync(handle_voice_extract, fields, path, pipeline, voice_dir)
        finally:
            if path and os.path.exists(path):
                os.remove(path)
        return JSONResponse(payload, status_code=code)

    return app
