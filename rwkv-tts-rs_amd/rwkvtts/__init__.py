"""rwkvtts -- MI355X-native RWKV-TTS hot path (host mirror of liuzl/rwkv-tts-rs's runtime,
sampler and batch-manager interfaces over the C-ABI in include/rwkvtts.h)."""
from . import _ffi  # noqa: F401
from ._ffi import (EOS_TOKEN, GLOBAL_TOKEN_OFFSET, HOP, N_GLOBAL, SAMPLE_RATE, SEMANTIC_LIMIT,  # noqa: F401
                   SPECIAL_TOKEN_OFFSET, TAG_0, TAG_1, TAG_2, RwkvTtsError)
from .properties import convert_standard_properties_to_tokens  # noqa: F401
from .runtime import (DynamicBatchConfig, DynamicBatchManager, LayeredRandomnessConfig, RnnInput,  # noqa: F401
                      RnnInputBatch, RnnOption, SamplerArgs, SharedRwkvRuntime, StdRng, TtsBatchRequest,
                      sample_logits_with_top_p_k)
from . import weights  # noqa: F401
