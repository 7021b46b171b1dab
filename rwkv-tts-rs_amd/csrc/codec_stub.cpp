// codec_stub.cpp -- placeholder entry points for the codec and mel rows (built later).
#include "common.h"
using namespace rwkvtts;
extern "C" {
int64_t rwkvtts_codec_blob_bytes(const rwkvtts_codec_dims*) { return -1; }
int rwkvtts_codec_synth_weights(const rwkvtts_codec_dims*, uint64_t, float*) { set_error("codec not built"); return RWKVTTS_EUNSUPPORTED; }
int rwkvtts_codec_create(int, const rwkvtts_codec_dims*, const float*, rwkvtts_codec**) { set_error("codec not built"); return RWKVTTS_EUNSUPPORTED; }
int rwkvtts_codec_destroy(rwkvtts_codec*) { return RWKVTTS_OK; }
int rwkvtts_codec_decode(rwkvtts_codec*, const int64_t*, int, const int64_t*, float*) { set_error("codec not built"); return RWKVTTS_EUNSUPPORTED; }
int rwkvtts_codec_decode_batch(rwkvtts_codec*, const int64_t* const*, const int*, const int64_t* const*, int, float* const*) { set_error("codec not built"); return RWKVTTS_EUNSUPPORTED; }
int rwkvtts_mel(int, const float*, int, float*, int*) { set_error("mel not built"); return RWKVTTS_EUNSUPPORTED; }
}
