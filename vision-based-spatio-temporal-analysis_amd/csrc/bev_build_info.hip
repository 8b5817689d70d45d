// bev_build_info.hip -- provenance of libbev_mi355x.so: the digest of the sources it was compiled from.
// The Makefile passes BEV_SRC_HASH = first 16 hex digits of sha256 over the library's sources and headers
// (SRCS then HDRS, in Makefile order); bev_native.source_hash() computes the same digest from the tree, so a
// loaded library can be checked against the sources next to it (__graft_entry__.build(), bench.py).
#include "../../include/bev_mi355x.h"

#ifndef BEV_SRC_HASH
#define BEV_SRC_HASH "unknown"
#endif

extern "C" const char *bev_build_source_hash(void) { return BEV_SRC_HASH; }
