"""Oracle mel restatement (src/tts_pipeline_fixes.rs:12-159): shapes and physical sanity (CPU)."""
import numpy as np

from rwkvtts import features


def test_frame_count_matches_reference_formula(oracle_mod):
    for n in (0, 1, 319, 320, 16000):
        assert oracle_mod.mel(np.zeros(n, np.float32)).shape == (128, features.n_frames(n))
    assert features.n_frames(16000) == 51


def test_silence_is_zero_and_tone_peaks_in_its_band(oracle_mod):
    assert not oracle_mod.mel(np.zeros(3200, np.float32)).any()
    t = np.arange(16000) / 16000.0
    m = oracle_mod.mel((0.5 * np.sin(2 * np.pi * 1000 * t)).astype(np.float32))
    band = int(np.argmax(m[:, 25]))
    # mel band of 1 kHz on the 2595*log10(1 + f/700) scale between 10 Hz and 8 kHz, 128 bands
    mel = lambda f: 2595 * np.log10(1 + f / 700)
    expect = (mel(1000) - mel(10)) / (mel(8000) - mel(10)) * 129 - 1
    assert abs(band - expect) <= 1.5
