"""Compile each HIP source for gfx950 with the resource-usage remarks and list every kernel's VGPRs and
scratch bytes per lane; exit 1 if any kernel spills to scratch. Usage: check_spills.py [files...]"""
import os
import re
import subprocess
import sys
import tempfile

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rwkv-tts-rs_amd", "csrc")


def usage(src):
    with tempfile.TemporaryDirectory() as td:
        out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=on",
                              "-c", src, "-o", os.path.join(td, "k.o"), "-Rpass-analysis=kernel-resource-usage"],
                             cwd=CSRC, capture_output=True, text=True).stderr
    res = {}
    for name, body in re.findall(r"Function Name: (\S+)(.*?)(?=Function Name:|\Z)", out, re.S):
        v = re.search(r"VGPRs: (\d+)", body)
        sc = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", body)
        res[name] = (int(v.group(1)) if v else -1, int(sc.group(1)) if sc else -1)
    return res


def main(files):
    bad = []
    for f in files:
        for k, (v, sc) in usage(f).items():
            if sc > 0:
                bad.append((f, k, v, sc))
            print(f"{f:16s} {v:4d} VGPRs {sc:5d} B scratch  {k[:90]}")
    if bad:
        print("SPILLS:", bad)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:] or ["lm_kernels.hip", "sampler.hip", "codec.hip", "mel.hip", "engine.hip"]))
