"""Sanitizer builds on the CPU (SURVEY §5's planned ASan/UBSan):

* the oracle's C restatement under AddressSanitizer + UndefinedBehaviorSanitizer, as one native
  executable (oracle/san_main.c, `make -C oracle san_check`) driving every entry point the tests
  reach through ctypes -- RNG, sampler on adversarial rows (ties, one-hot, -inf, 77,923 wide), the
  RWKV-7 forward and the three phase controllers on a tiny model, Int8 quantisation, mel on edge
  lengths, the codec on tiny dims;
* csrc/manager.cpp compiled UNCHANGED under ThreadSanitizer against the stub engine of
  tests/native/stub/engine.h (ROCm's clang++: gcc 11's TSan does not intercept
  pthread_cond_clockwait and reports condition_variable::wait_for as a double lock), driven by
  tests/native/manager_tsan_main.cpp: 8 submitter / waiter threads over 3 engines, recoverable engine
  faults, destroy with blocked waiters and queued requests, an engine that dies.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

from rwkvtts import codec
from rwkvtts import weights as W

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/lib/llvm/bin/clang++"


def test_oracle_under_asan_ubsan(tmp_path):
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "san_check"])
    blob = tmp_path / "model.bin"
    W.synth_blob(W.DIMS_TINY, seed=7).tofile(blob)
    d = codec.CODEC_DIMS_TINY
    dims = tmp_path / "codec_dims.bin"
    dims.write_bytes(bytes(codec.make_codec_dims(d)))
    cw = tmp_path / "codec_w.bin"
    np.asarray(codec.synth_codec_blob(d), dtype=np.float32).tofile(cw)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1",
               OMP_NUM_THREADS="2")
    out = subprocess.run([os.path.join(ROOT, "oracle", "san_check"), str(blob), str(dims), str(cw)],
                         capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0 and "san_check: ok" in out.stdout, (out.stdout[-2000:], out.stderr[-4000:])
    assert "runtime error" not in out.stderr and "AddressSanitizer" not in out.stderr, out.stderr[-4000:]


@pytest.mark.skipif(not os.path.exists(CLANG), reason="ROCm clang++ (TSan runtime) not present")
def test_manager_under_tsan(tmp_path):
    src = os.path.join(ROOT, "rwkv-tts-rs_amd", "csrc", "manager.cpp")
    stub = os.path.join(ROOT, "tests", "native", "stub")
    # manager.cpp includes "engine.h" from its own directory: build a copy beside the stub engine
    shutil.copy(src, tmp_path / "manager.cpp")
    eh = open(os.path.join(stub, "engine.h")).read().replace('"../../../include/rwkvtts.h"', '"rwkvtts.h"')
    (tmp_path / "engine.h").write_text(eh)
    exe = tmp_path / "manager_tsan"
    subprocess.check_call([CLANG, "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-Wno-enum-compare",
                           "-I", stub, "-I", os.path.join(ROOT, "include"), "-I", str(tmp_path), "-o", str(exe),
                           os.path.join(ROOT, "tests", "native", "manager_tsan_main.cpp"), str(tmp_path / "manager.cpp"),
                           "-ldl", "-lpthread"])
    env = dict(os.environ, RWKVTTS_MANAGER_NO_RCCL="1", TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    for k in ("STUB_FAIL_EVERY", "STUB_DEAD_ENGINE", "STUB_EXPECT_RCCL"):
        env.pop(k, None)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0 and "manager_tsan: ok" in out.stdout, (out.stdout[-2000:], out.stderr[-6000:])
    assert "ThreadSanitizer" not in out.stderr, out.stderr[-6000:]
    # the multi-rank RCCL weight broadcast (only ever run with one device): the
    # manager over four distinct devices with RCCL enabled, against the host-memory RCCL stand-in
    # (tests/native/stub/rccl/stub_rccl.cpp, found by the manager's dlopen of librccl.so.1): one
    # ncclCommInitAll over the four devices, four broadcasts in one group, every engine's copy checked
    libdir = tmp_path / "rccl"
    libdir.mkdir()
    subprocess.check_call([CLANG, "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-shared", "-fPIC",
                           "-I", os.path.join(stub, "rccl"), "-o", str(libdir / "librccl.so.1"),
                           os.path.join(stub, "rccl", "stub_rccl.cpp")])
    env2 = dict(env, STUB_EXPECT_RCCL="1", LD_LIBRARY_PATH=str(libdir) + ":" + os.environ.get("LD_LIBRARY_PATH", ""))
    env2.pop("RWKVTTS_MANAGER_NO_RCCL")
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env2)
    assert out.returncode == 0 and "manager_tsan: ok" in out.stdout, (out.stdout[-2000:], out.stderr[-6000:])
    assert "ThreadSanitizer" not in out.stderr, out.stderr[-6000:]
    assert "stub_rccl: grouped broadcast of 4096 bytes to 4 ranks" in out.stderr, out.stderr[-3000:]
