"""The reference's own unit tests on this path, restated against the host mirrors:
src/lightweight_tts_pipeline.rs:66-140 (pipeline args defaults / custom / clone, cross-lingual
process_text_zero_shot) and src/voice_feature_manager.rs:495-545 (save / load / list / rename /
delete). src/streaming_inference.rs:422-450 is covered by tests/test_streaming.py."""
import copy

from rwkvtts.pipeline import LightweightTtsPipeline, LightweightTtsPipelineArgs
from rwkvtts.voices import VoiceFeatureManager


def test_pipeline_args_default():
    a = LightweightTtsPipelineArgs()
    assert a.prompt_text == "" and a.ref_audio_path == "" and a.text == ""
    assert a.temperature == 1.0 and a.top_p == 0.90 and a.top_k == 0 and a.max_tokens == 8000
    assert (a.age, a.gender, a.emotion, a.pitch, a.speed) == ("youth-adult", "female", "NEUTRAL", "medium", "medium")
    assert not a.zero_shot and not a.validate
    assert a.seed is None and a.voice_id is None
    assert a.voice_global_tokens is None and a.voice_semantic_tokens is None


def test_pipeline_args_custom():
    a = LightweightTtsPipelineArgs(prompt_text="这是提示文本", ref_audio_path="/path/to/audio.wav",
                                   text="这是要合成的文本", zero_shot=True)
    assert (a.prompt_text, a.ref_audio_path, a.text, a.zero_shot) == (
        "这是提示文本", "/path/to/audio.wav", "这是要合成的文本", True)


def test_pipeline_args_clone():
    a = LightweightTtsPipelineArgs(prompt_text="测试克隆", ref_audio_path="/test/path.wav")
    b = copy.deepcopy(a)
    assert (a.prompt_text, a.ref_audio_path) == (b.prompt_text, b.ref_audio_path)


def test_process_text_zero_shot():
    # cross-lingual mode: the prompt text is not prepended
    assert LightweightTtsPipeline.process_text_zero_shot("用户文本", "提示文本") == "用户文本"


def test_voice_feature_manager(tmp_path):
    m = VoiceFeatureManager(str(tmp_path))
    vid = m.save_voice_feature("测试音色", "这是一个测试音色", [1, 2, 3, 4, 5], [6, 7, 8, 9, 10], 5.0, 16000)
    f = m.load_voice_feature(vid)
    assert f.name == "测试音色" and f.global_tokens == [1, 2, 3, 4, 5]
    voices = m.list_voices()
    assert len(voices) == 1 and voices[0].name == "测试音色"
    m.rename_voice(vid, "新名称")
    assert m.load_voice_feature(vid).name == "新名称"
    after = m.list_voices()
    assert len(after) == 1 and after[0].name == "新名称"
    m.delete_voice(vid)
    assert len(m.list_voices()) == 0
