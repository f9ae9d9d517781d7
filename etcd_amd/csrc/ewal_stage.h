// ewal_stage.h -- staging of host bytes into a ctx's device buffer, shared by
// the two translation units of libewal.so (ewal_api.hip implements it,
// ewal_host.cpp's OpenAtIndex/ReadAll pipeline uses it).  Exported, but not
// part of the public C ABI (include/ewal.h).
#ifndef EWAL_STAGE_H
#define EWAL_STAGE_H
#include <stdint.h>
#include "../../include/ewal.h"

extern "C" {
/* size the ctx's staging buffer for len bytes */
int ewal_stage_begin(ewal_ctx *ctx, uint64_t len);
/* host -> staging buffer [off, off + n), asynchronous on the ctx stream; h
 * must stay unchanged until ewal_stage_readall returns */
int ewal_stage_put(ewal_ctx *ctx, uint64_t off, const void *h, uint64_t n);
/* wait for the queued puts (their host bytes may be released afterwards) */
int ewal_stage_sync(ewal_ctx *ctx);
/* (*WAL).ReadAll over the staged len bytes (stream-ordered after the puts) */
int ewal_stage_readall(ewal_ctx *ctx, uint64_t len, uint64_t ri, ewal_result *out);
}
#endif
