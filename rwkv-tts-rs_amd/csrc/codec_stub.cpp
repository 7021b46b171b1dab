// codec_stub.cpp -- placeholder entry point for the zero-shot mel row (built later).
#include "common.h"
using namespace rwkvtts;
extern "C" {
int rwkvtts_mel(int, const float*, int, float*, int*) { set_error("mel not built"); return RWKVTTS_EUNSUPPORTED; }
}
