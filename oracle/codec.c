/* codec.c -- TEST INFRASTRUCTURE (see oracle.h). Placeholder until the codec row is built. */
#include "oracle.h"
int oracle_codec_decode(const rwkvtts_codec_dims* d, const float* w, const int64_t* s, int T, const int64_t* g, float* pcm) { (void)d; (void)w; (void)s; (void)T; (void)g; (void)pcm; return -4; }
