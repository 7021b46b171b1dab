// TEST INFRASTRUCTURE: the declarations manager.cpp takes decltype of (stub_rccl.cpp implements them
// on host memory for the multi-rank broadcast test)
#pragma once
#include <stddef.h>
typedef void* hipStream_t;
typedef struct ncclComm* ncclComm_t;
typedef enum { ncclSuccess = 0 } ncclResult_t;
typedef enum { ncclUint8 = 1 } ncclDataType_t;
#ifdef __cplusplus
extern "C" {
#endif
ncclResult_t ncclCommInitAll(ncclComm_t* comms, int n, const int* devs);
ncclResult_t ncclCommDestroy(ncclComm_t comm);
ncclResult_t ncclBroadcast(const void* s, void* r, size_t n, ncclDataType_t t, int root, ncclComm_t c, hipStream_t st);
ncclResult_t ncclGroupStart(void);
ncclResult_t ncclGroupEnd(void);
const char* ncclGetErrorString(ncclResult_t r);
#ifdef __cplusplus
}
#endif
