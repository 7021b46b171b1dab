"""Generates tests/golden/properties_golden.json by running the reference's own compiled helper
参考/python/__pycache__/properties_util.cpython-310.pyc (read-only, imported in this container
only; the GPU box never needs it). Output: input attribute tuples -> the reference's prompt
string ("SPCT_<n>..." ids in the Python model's id space)."""
import importlib.machinery
import importlib.util
import itertools
import json
import os

PYC = "/root/reference/参考/python/__pycache__/properties_util.cpython-310.pyc"


def main():
    loader = importlib.machinery.SourcelessFileLoader("properties_util", PYC)
    spec = importlib.util.spec_from_loader("properties_util", loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    ages = ["child", "teenager", "youth-adult", "middle-aged", "elderly", "bogus"]
    genders = ["female", "male", "other"]
    emotions = ["NEUTRAL", "HAPPY", "SAD", "ANGRY", "WHISPER", "CONTEMPT", "nope"]
    pitches = ["low_pitch", "medium_pitch", "high_pitch", "very_high_pitch", "low", "medium"]
    speeds = ["very_slow", "slow", "medium", "fast", "very_fast", "x"]
    cases = []
    for a, g, e, p, s in itertools.product(ages, genders, emotions, pitches, speeds):
        try:
            out = mod.convert_standard_properties_to_tokens(a, g, e, p, s)
        except Exception as ex:  # record the reference's behaviour on unknown inputs too
            out = "ERROR:" + type(ex).__name__
        cases.append({"age": a, "gender": g, "emotion": e, "pitch": p, "speed": s, "out": out})
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "properties_golden.json")
    json.dump({"source": PYC.replace("/root/reference/", ""), "cases": cases}, open(path, "w"))
    print(len(cases), cases[0])


if __name__ == "__main__":
    main()
