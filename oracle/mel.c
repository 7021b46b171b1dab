/* mel.c -- TEST INFRASTRUCTURE (see oracle.h). Placeholder until the mel row is built. */
#include "oracle.h"
int oracle_mel(const float* wav, int n, float* mel, int* n_frames) { (void)wav; (void)n; (void)mel; (void)n_frames; return -4; }
