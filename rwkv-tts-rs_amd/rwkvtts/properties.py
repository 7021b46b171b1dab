"""Attribute -> prompt tokens: src/properties_util.rs:5-98 (TTS_SPECIAL_TOKEN_OFFSET = 77823;
order age, gender, emotion, pitch, speed; unknown strings fall back to 15/46/26/7/3)."""
TTS_SPECIAL_TOKEN_OFFSET = 77823
SPEED_MAP = {"very_slow": 1, "slow": 2, "medium": 3, "fast": 4, "very_fast": 5}
PITCH_MAP = {"low_pitch": 6, "medium_pitch": 7, "high_pitch": 8, "very_high_pitch": 9}
AGE_MAP = {"child": 13, "teenager": 14, "youth-adult": 15, "middle-aged": 16, "elderly": 17}
GENDER_MAP = {"female": 46, "male": 47}
EMOTION_MAP = {k: 21 + i for i, k in enumerate([
    "UNKNOWN", "NEUTRAL", "ANGRY", "HAPPY", "SAD", "FEARFUL", "DISGUSTED", "SURPRISED", "SARCASTIC",
    "EXCITED", "SLEEPY", "CONFUSED", "EMPHASIS", "LAUGHING", "SINGING", "WORRIED", "WHISPER", "ANXIOUS",
    "NO-AGREEMENT", "APOLOGETIC", "CONCERNED", "ENUNCIATED", "ASSERTIVE", "ENCOURAGING", "CONTEMPT"])}


def convert_standard_properties_to_tokens(age, gender, emotion, pitch, speed):
    o = TTS_SPECIAL_TOKEN_OFFSET
    return [o, o + AGE_MAP.get(age, 15), o + GENDER_MAP.get(gender, 46), o + EMOTION_MAP.get(emotion, 26),
            o + PITCH_MAP.get(pitch, 7), o + SPEED_MAP.get(speed, 3)]
