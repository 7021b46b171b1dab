"""text -> tokens -> GPU scheduler -> GPU vocoder -> PCM (LightweightTtsPipeline.generate_speech,
src/lightweight_tts_pipeline.rs:733-852) and the /api/tts handler on top, against the oracle:
the tokenizer's ids feed the oracle's serial controller, its tokens the oracle vocoder."""
import base64
import json

import numpy as np
import pytest

import rwkvtts
from rwkvtts import codec as CC
from rwkvtts import server as SV
from rwkvtts import weights as W
from rwkvtts.pipeline import LightweightTtsPipeline, LightweightTtsPipelineArgs
from rwkvtts.tokenizer import Tokenizer
from test_tokenizer import VOCAB
from helpers import to_struct

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def stack():
    import oracle
    blob = W.synth_blob(W.DIMS_TINY, seed=99)
    tok = Tokenizer(VOCAB)
    m = rwkvtts.DynamicBatchManager(blob, devices=[0], max_slots=4, token_chunk_size=64, tokenizer=tok)
    cd = CC.CODEC_DIMS_TINY
    cw = CC.synth_codec_blob(cd, seed=11)
    voc = CC.BiCodecDetokenizer(cw, cd)
    yield LightweightTtsPipeline(m, voc), oracle.Model(blob), tok, cd, cw
    m.close()
    voc.close()


def _oracle_pcm(om, cd, cw, req):
    import oracle
    q, keep = to_struct(req)
    g, s, _ = om.generate(q)
    return g, s, oracle.codec_decode(CC.make_codec_dims(cd), cw, s, g)


def test_generate_speech_matches_oracle(stack):
    pipe, om, tok, cd, cw = stack
    args = LightweightTtsPipelineArgs(text="Hello world, this is RWKV speaking.", seed=12, max_tokens=40)
    pcm = pipe.generate_speech(args)
    req = pipe._request(args)
    assert req.text_tokens == tok.encode(args.text)
    g, s, ref = _oracle_pcm(om, cd, cw, req)
    assert pcm.shape == (len(s) * 320,) and pcm.size > 0
    assert np.abs(pcm - ref).max() <= 5e-4  # test_gpu_codec.py's PCM tolerance


def test_api_tts_end_to_end(stack):
    pipe, om, tok, cd, cw = stack
    code, body = SV.handle_tts_json(json.dumps({"text": "你好，世界！", "seed": 5, "gender": "female"}), pipe)
    assert code == 200 and body["success"]
    wav = base64.b64decode(body["audio_base64"])
    args = LightweightTtsPipelineArgs(text="你好，世界！", seed=5, gender="female", top_k=100, max_tokens=8000)
    g, s, ref = _oracle_pcm(om, cd, cw, pipe._request(args))
    assert len(wav) == 48 + 2 * len(s) * 320
    pcm16 = np.frombuffer(wav[48:], dtype="<i2")
    ref16 = np.frombuffer(SV.convert_samples_to_wav(ref)[48:], dtype="<i2")
    mx = float(np.abs(ref).max())
    gain = 1.0 / mx if mx > 1 else min(0.8 / mx, 10.0)
    # PCM tolerance 5e-4 through the peak-normalisation gain, +1 for the truncation step
    assert np.abs(pcm16.astype(int) - ref16.astype(int)).max() <= 5e-4 * gain * 32767 * 1.01 + 1


def test_batch_and_silence(stack):
    pipe, om, tok, cd, cw = stack
    outs = pipe.generate_speech_batch([LightweightTtsPipelineArgs(text="one", seed=1, max_tokens=12),
                                       LightweightTtsPipelineArgs(text="emoji \U0001F600", seed=2),
                                       LightweightTtsPipelineArgs(text="three", seed=3, max_tokens=9)])
    assert outs[1].size == 0 and outs[0].size > 0 and outs[2].size > 0
    out = pipe.generate_speech(LightweightTtsPipelineArgs(text="emoji \U0001F600"))
    assert out.shape == (16000,) and not out.any()
