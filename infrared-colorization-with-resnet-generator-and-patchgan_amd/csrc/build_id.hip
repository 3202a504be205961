// irgan_build_id: the source id libirgan.so was built from (include/irgan.h).
// IRGAN_SOURCE_ID is a hash of csrc/*.hip, csrc/*.h and include/irgan.h computed by
// _build.source_id() and passed as a -D flag; _lib.load() refuses a library whose id does
// not match the tree it is loaded from, so a stale binary cannot stand in for HEAD.
#include "common.h"

#ifndef IRGAN_SOURCE_ID
#error "IRGAN_SOURCE_ID must be defined by the build (_build.py)"
#endif

extern "C" IRGAN_API int irgan_build_id(char* buf, int32_t len) {
  const char* id = IRGAN_SOURCE_ID;
  int32_t n = 0;
  if (!buf || len <= 0) return IRGAN_EINVAL;
  while (id[n] && n < len - 1) { buf[n] = id[n]; ++n; }
  buf[n] = 0;
  return id[n] ? IRGAN_EINVAL : 0;
}
