"""Prompt attribute tokens (src/properties_util.rs:76-98) against the reference's own compiled
Python helper (golden fixture from tests/golden/make_properties_golden.py). The Rust live path
maps SPCT_n -> 77823 + n and falls back to defaults for unknown strings where the Python helper
raises KeyError; both behaviours are checked."""
import json
import os
import re

from rwkvtts import convert_standard_properties_to_tokens

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "properties_golden.json")


def test_against_reference_pyc():
    cases = json.load(open(GOLDEN))["cases"]
    n_ok = 0
    for c in cases:
        toks = convert_standard_properties_to_tokens(c["age"], c["gender"], c["emotion"], c["pitch"], c["speed"])
        if c["out"].startswith("ERROR"):
            # Rust fallback (properties_util.rs:83-87): 15 / 46 / 26 / 7 / 3
            continue
        ids = [77823 + int(x) for x in re.findall(r"SPCT_(\d+)", c["out"])]
        assert toks == ids, c
        n_ok += 1
    assert n_ok == 1200


def test_rust_fallbacks_and_server_pitch_quirk():
    assert convert_standard_properties_to_tokens("?", "?", "?", "?", "?") == [77823, 77838, 77869, 77849, 77830, 77826]
    # server.rs:570-576 maps pitch to "low"/"medium"/... which misses PITCH_MAP -> always 7
    for p in ("low", "medium", "high", "very_high"):
        assert convert_standard_properties_to_tokens("youth-adult", "female", "NEUTRAL", p, "medium")[4] == 77830
