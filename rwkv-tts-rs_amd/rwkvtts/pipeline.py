"""End-to-end text -> PCM: host mirror of `LightweightTtsPipeline` (src/lightweight_tts_pipeline.rs).

generate_speech (:733-852): text (+ attribute strings, or a voice's reference tokens) -> property
tokens (:162-193) -> DynamicBatchManager.generate_tts (which tokenises the text,
dynamic_batch_manager.rs:512-515) -> BiCodec decode (:606-622) -> f32 PCM @ 16 kHz; an empty
generation (a failed request) becomes one second of silence (:828-830).
generate_speech_batch (:855-1000): the same for a list of args through generate_tts_batch and
decode_audio_batch (a failed item decodes to an empty array there, as the reference's
spawn_blocking tasks return vec![]).

The voice store lookup by voice_id inside the pipeline (`VoiceFeatureManager::new("./raf")`,
:751) goes through `voices.VoiceFeatureManager` on `raf_dir` (the server passes the
tokens directly instead).
"""
import dataclasses
import os
from typing import List, Optional, Sequence

import numpy as np

from .properties import convert_standard_properties_to_tokens
from .runtime import LayeredRandomnessConfig, SamplerArgs, TtsBatchRequest

SAMPLE_RATE = 16000


@dataclasses.dataclass
class LightweightTtsPipelineArgs:  # :18-65 (Default)
    text: str = ""
    prompt_text: str = ""
    ref_audio_path: str = ""
    temperature: float = 1.0
    top_p: float = 0.90
    top_k: int = 0
    max_tokens: int = 8000
    age: str = "youth-adult"
    gender: str = "female"
    emotion: str = "NEUTRAL"
    pitch: str = "medium"
    speed: str = "medium"
    zero_shot: bool = False
    validate: bool = False
    seed: Optional[int] = None
    voice_id: Optional[str] = None
    voice_global_tokens: Optional[List[int]] = None
    voice_semantic_tokens: Optional[List[int]] = None


class LightweightTtsPipeline:
    """manager: rwkvtts.DynamicBatchManager (with a tokenizer); codec: BiCodecDetokenizer."""

    def __init__(self, manager, codec, raf_dir: str = "./raf", reference_tokenizer=None):
        self.manager = manager
        self.codec = codec
        self.raf_dir = raf_dir
        # zero-shot from a reference audio file needs the BiCodecTokenize / wav2vec2 encoders,
        # whose graphs are not available; a callable (path -> (global, semantic))
        # may be supplied
        self.reference_tokenizer = reference_tokenizer

    # ---- text / attribute handling (:148-193)
    @staticmethod
    def process_text(text: str) -> str:
        return text

    @staticmethod
    def process_text_zero_shot(text: str, _prompt_text: str) -> str:
        """Cross-lingual cloning: the reference prompt text is ignored (:157-160)."""
        return text

    @staticmethod
    def generate_property_tokens(args: LightweightTtsPipelineArgs) -> List[int]:
        if (args.voice_global_tokens is not None and args.voice_semantic_tokens is not None) or args.zero_shot:
            return []
        return convert_standard_properties_to_tokens(args.age, args.gender, args.emotion, args.pitch, args.speed)

    def _voice_tokens(self, voice_id: str):
        """VoiceFeatureManager::new(raf_dir).get_voice_tokens (:751-760; checksum verified)."""
        from .voices import VoiceFeatureManager
        if getattr(self, "_voices", None) is None:
            self._voices = VoiceFeatureManager(self.raf_dir)
        return self._voices.get_voice_tokens(voice_id)

    def process_reference_audio(self, ref_audio_path: str):
        if not ref_audio_path or not os.path.exists(ref_audio_path):
            raise FileNotFoundError(f"reference audio not found: {ref_audio_path}")
        if self.reference_tokenizer is None:
            raise NotImplementedError("reference-audio tokenisation needs the BiCodecTokenize encoder")
        return self.reference_tokenizer(ref_audio_path)

    def _prompt_parts(self, args: LightweightTtsPipelineArgs):
        """(property tokens, ref global, ref semantic) with the reference's precedence (:747-789)."""
        have_voice = args.voice_global_tokens is not None and args.voice_semantic_tokens is not None
        if args.voice_id is not None:
            try:
                g, s = self._voice_tokens(args.voice_id)
                return [], g, s
            except (OSError, KeyError, ValueError):
                pass  # fall through to the directly supplied tokens / attributes
        if have_voice:
            return [], list(args.voice_global_tokens), list(args.voice_semantic_tokens)
        if args.zero_shot:
            g, s = self.process_reference_audio(args.ref_audio_path)
            return [], g, s
        return self.generate_property_tokens(args), None, None

    def _request(self, args: LightweightTtsPipelineArgs) -> TtsBatchRequest:
        text = self.process_text_zero_shot(args.text, args.prompt_text) if args.zero_shot else self.process_text(args.text)
        props, rg, rs = self._prompt_parts(args)
        sargs = SamplerArgs(temperature=args.temperature, top_p=args.top_p, top_k=args.top_k,
                            max_tokens=args.max_tokens, seed=args.seed, voice_fidelity=0.8,
                            layered_randomness=LayeredRandomnessConfig(), token_chunk_size=512)
        return TtsBatchRequest(self.manager._tokens(text), props, rg, rs, sargs, args.voice_id)

    def generate_speech(self, args: LightweightTtsPipelineArgs) -> np.ndarray:
        try:
            req = self._request(args)
        except ValueError:  # untokenisable text: the request fails -> empty result
            req = None
        g, s = self.manager.generate_tts_batch([req])[0] if req is not None else ([], [])
        if not g and not s:
            return np.zeros(SAMPLE_RATE, dtype=np.float32)  # :828-830
        return self.codec.decode_audio(g, s)

    def generate_speech_batch(self, batch_args: Sequence[LightweightTtsPipelineArgs]) -> List[np.ndarray]:
        reqs, idx = [], []
        for i, a in enumerate(batch_args):
            try:
                reqs.append(self._request(a))
                idx.append(i)
            except ValueError:
                pass
        res = self.manager.generate_tts_batch(reqs) if reqs else []
        results = [([], [])] * len(batch_args)
        for i, r in zip(idx, res):
            results[i] = r
        return self.codec.decode_audio_batch(results)
