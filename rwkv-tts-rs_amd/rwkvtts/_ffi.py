"""ctypes binding of include/rwkvtts.h (the C-ABI drop-in boundary).

This is the Python twin of the Rust `extern "C"` block in INTEGRATION.md: same structs, same
entry points. The product library is loaded from this directory (built in-tree by
`make -C rwkv-tts-rs_amd/csrc`); there is no fallback -- a missing library is an error.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# RWKVTTS_LIB: an alternative build of the same library (A/B timing tools only)
LIB_PATH = os.environ.get("RWKVTTS_LIB") or os.path.join(_HERE, "librwkvtts.so")


def build_id() -> str:
    """Identity of the in-tree library's build: sha256 over the sources it is built from
    (csrc/*.hip, *.cpp, *.h, the Makefile and include/*.h, in name order), first 16 hex digits.
    Profile summaries under profiles/ carry it (tools/), so bench.py cites only summaries that were
    measured on the library it runs."""
    import glob
    import hashlib
    csrc = os.path.join(_HERE, "..", "csrc")
    inc = os.path.join(_HERE, "..", "..", "include")
    files = sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.cpp")) +
                   glob.glob(os.path.join(csrc, "*.h")) + [os.path.join(csrc, "Makefile")] +
                   glob.glob(os.path.join(inc, "*.h")), key=os.path.basename)
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]

EOS_TOKEN = 8192
TAG_0, TAG_1, TAG_2 = 8193, 8194, 8195
GLOBAL_TOKEN_OFFSET = 8196
SPECIAL_TOKEN_OFFSET = 77823
N_GLOBAL = 32
SEMANTIC_LIMIT = 2048
HOP = 320
SAMPLE_RATE = 16000

OK, EINVAL, EHIP, ENOMEM, EUNSUPPORTED, EBUSY, ECLOSED = 0, -1, -2, -3, -4, -5, -6
MAX_ENGINES = 16
DTYPE_BF16, DTYPE_F16 = 0, 1
OPT_LAST, OPT_FULL = 0, 1


class Dims(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "n_layer", "n_embd", "head_size", "n_ffn", "n_vocab", "d_decay", "d_aaa", "d_mv", "d_gate")]


class EngineDesc(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("max_slots", ctypes.c_int32),
                ("token_chunk_size", ctypes.c_int32), ("use_graphs", ctypes.c_int32),
                ("wkv_variant", ctypes.c_int32), ("quant_layers", ctypes.c_int32),
                ("quant_type", ctypes.c_int32), ("forms", ctypes.c_uint32)]


# rwkvtts_engine_desc.forms (include/rwkvtts.h RWKVTTS_FORM_*): each bit switches one fused decode form
# back to the launches it replaces (bitwise-equal outputs; verification and A/B timing only)
FORM_SEPARATE_ATT, FORM_SEPARATE_FFN, FORM_LN_ROWS, FORM_SLAB_HANDOFF = 1, 2, 4, 8
FORM_SEPARATE_LNOUT, FORM_SEPARATE_EMBED, FORM_EXACT_SAMPLER = 16, 32, 64
# codec weight paths and forms (RWKVTTS_CODEC_WEIGHTS_* / RWKVTTS_CODEC_FORM_*)
CODEC_WEIGHTS_AUTO, CODEC_WEIGHTS_BF16, CODEC_WEIGHTS_HILO = 0, 1, 2
CODEC_FORM_SEPARATE_RESUNIT, CODEC_FORM_CHANNEL_LAST = 1, 2


QUANT_NONE, QUANT_INT8, QUANT_NF4, QUANT_SF4 = 0, 1, 2, 3


class Input(ctypes.Structure):
    _fields_ = [("slot", ctypes.c_int32), ("tokens", ctypes.POINTER(ctypes.c_uint32)),
                ("n_tokens", ctypes.c_int32), ("option", ctypes.c_int32)]


class Rng(ctypes.Structure):
    _fields_ = [("key", ctypes.c_uint32 * 8), ("draw_index", ctypes.c_uint64)]


class SampleArgs(ctypes.Structure):
    _fields_ = [("temperature", ctypes.c_float), ("top_p", ctypes.c_float),
                ("top_k", ctypes.c_int32), ("forbid_token", ctypes.c_int32)]


class Request(ctypes.Structure):
    _fields_ = [("text_tokens", ctypes.POINTER(ctypes.c_int32)), ("n_text", ctypes.c_int32),
                ("property_tokens", ctypes.POINTER(ctypes.c_int32)), ("n_property", ctypes.c_int32),
                ("ref_global", ctypes.POINTER(ctypes.c_int32)), ("n_ref_global", ctypes.c_int32),
                ("ref_semantic", ctypes.POINTER(ctypes.c_int32)), ("n_ref_semantic", ctypes.c_int32),
                ("has_seed", ctypes.c_int32), ("seed", ctypes.c_uint64),
                ("max_tokens", ctypes.c_int32), ("fixed_semantic", ctypes.c_int32),
                ("greedy", ctypes.c_int32), ("layered_set", ctypes.c_int32),
                ("use_independent_seeds", ctypes.c_int32), ("global_seed_offset", ctypes.c_uint64),
                ("semantic_seed_offset", ctypes.c_uint64)]


class Result(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("n_global", ctypes.c_int32),
                ("n_semantic", ctypes.c_int32), ("global_tokens", ctypes.c_int32 * N_GLOBAL),
                ("semantic_tokens", ctypes.POINTER(ctypes.c_int32))]


class Stats(ctypes.Structure):
    _fields_ = [("steps", ctypes.c_int64), ("prefill_steps", ctypes.c_int64),
                ("decode_ms", ctypes.c_double), ("prefill_ms", ctypes.c_double),
                ("sample_ms", ctypes.c_double), ("decode_rows", ctypes.c_int64),
                ("profile_kernel_count", ctypes.c_int32), ("persistent", ctypes.c_int32)]


class ManagerDesc(ctypes.Structure):
    _fields_ = [("n_engines", ctypes.c_int32), ("devices", ctypes.c_int32 * MAX_ENGINES),
                ("engine", EngineDesc), ("max_batch_size", ctypes.c_int32),
                ("collect_timeout_ms", ctypes.c_int32)]


class ManagerStats(ctypes.Structure):
    _fields_ = [("submitted", ctypes.c_int64), ("completed", ctypes.c_int64), ("batches", ctypes.c_int64),
                ("served", ctypes.c_int64 * MAX_ENGINES), ("max_active", ctypes.c_int64 * MAX_ENGINES),
                ("steps", ctypes.c_int64 * MAX_ENGINES), ("bcast_ranks", ctypes.c_int32),
                ("bcast_rccl", ctypes.c_int32), ("bcast_ms", ctypes.c_double),
                ("waiters", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("persistent", ctypes.c_int32 * MAX_ENGINES)]


class CodecDims(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "codebook_size", "codebook_dim", "latent_dim", "n_global", "fsq_levels", "fsq_dims",
        "spk_dim", "prenet_dim", "prenet_inter", "prenet_layers", "dec_channels", "n_up")] + [
        ("up_rates", ctypes.c_int32 * 4), ("up_kernels", ctypes.c_int32 * 4)]


# Every symbol include/rwkvtts.h declares (checked by tests/test_abi.py against the header).
EXPORTS = {
    "rwkvtts_synth_weights": (ctypes.c_int, [ctypes.POINTER(Dims), ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p]),
    "rwkvtts_engine_create": (ctypes.c_int, [ctypes.POINTER(EngineDesc), ctypes.c_void_p, ctypes.c_size_t,
                                             ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "rwkvtts_engine_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "rwkvtts_last_error": (ctypes.c_char_p, []),
    "rwkvtts_engine_dims": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Dims)]),
    "rwkvtts_state_floats": (ctypes.c_int64, [ctypes.c_void_p]),
    "rwkvtts_slot_reset": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "rwkvtts_slot_read": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "rwkvtts_slot_write": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "rwkvtts_infer": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Input), ctypes.c_int, ctypes.c_int,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "rwkvtts_rng_seed_from_u64": (None, [ctypes.c_uint64, ctypes.POINTER(Rng)]),
    "rwkvtts_sample": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                      ctypes.POINTER(SampleArgs), ctypes.c_void_p, ctypes.c_void_p]),
    "rwkvtts_generate_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Request), ctypes.c_int,
                                              ctypes.POINTER(Result)]),
    "rwkvtts_manager_create": (ctypes.c_int, [ctypes.POINTER(ManagerDesc), ctypes.c_void_p, ctypes.c_size_t,
                                              ctypes.POINTER(ctypes.c_void_p)]),
    "rwkvtts_manager_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "rwkvtts_manager_submit": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Request),
                                              ctypes.POINTER(ctypes.c_uint64)]),
    "rwkvtts_manager_wait": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(Result)]),
    "rwkvtts_manager_generate_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Request), ctypes.c_int,
                                                      ctypes.POINTER(Result)]),
    "rwkvtts_manager_get_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ManagerStats)]),
    "rwkvtts_get_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Stats)]),
    "rwkvtts_set_profiling": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    # test hook (tests/test_gpu_advance.py): the decode-step sampler on caller-given rows
    "rwkvtts_debug_advance": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_void_p]),
    "rwkvtts_profile_entry": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                             ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double)]),
    "rwkvtts_codec_blob_bytes": (ctypes.c_int64, [ctypes.POINTER(CodecDims)]),
    "rwkvtts_codec_synth_weights": (ctypes.c_int, [ctypes.POINTER(CodecDims), ctypes.c_uint64, ctypes.c_void_p]),
    "rwkvtts_codec_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(CodecDims), ctypes.c_void_p,
                                            ctypes.POINTER(ctypes.c_void_p)]),
    "rwkvtts_codec_create_ex": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(CodecDims), ctypes.c_void_p,
                                               ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "rwkvtts_codec_set_forms": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32]),
    "rwkvtts_codec_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "rwkvtts_codec_decode": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                            ctypes.c_void_p]),
    "rwkvtts_codec_decode_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "rwkvtts_codec_set_profiling": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "rwkvtts_codec_profile_count": (ctypes.c_int, [ctypes.c_void_p]),
    "rwkvtts_codec_profile_entry": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                                   ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double)]),
    "rwkvtts_tokenizer_create": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]),
    "rwkvtts_tokenizer_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "rwkvtts_tokenizer_encode": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p,
                                                ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
    "rwkvtts_tokenizer_decode": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                                ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
    "rwkvtts_tokenizer_vocab_size": (ctypes.c_int64, [ctypes.c_void_p]),
    "rwkvtts_mel": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                   ctypes.POINTER(ctypes.c_int)]),
}

_lib = None


def lib():
    """Load librwkvtts.so (raises if it was not built: the product has no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `make -C rwkv-tts-rs_amd/csrc` "
                               "(the HIP extension is required; there is no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in EXPORTS.items():
            if os.environ.get("RWKVTTS_LIB") and not hasattr(L, name):
                continue  # (an A/B build of an earlier revision: entry points it predates stay unbound)
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


class RwkvTtsError(RuntimeError):
    def __init__(self, rc, where):
        self.code = rc
        msg = lib().rwkvtts_last_error()
        super().__init__(f"{where} failed ({rc}): {msg.decode() if msg else ''}")
        self.rc = rc


def check(rc, where):
    if rc != OK:
        raise RwkvTtsError(rc, where)
    return rc
