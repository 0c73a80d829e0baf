// Provenance of the built library (include/shine_gpu.h shine_build_id): a hash of every source file the library is
// built from and the git head at build time, compiled in by the Makefile, so a stale libshine_gpu.so is visible in the
// bench line, in smoke() and to tests/test_capi.py (which recomputes the hash over the tree).
#include "../../include/shine_gpu.h"

#ifndef SHINE_SRC_HASH
#define SHINE_SRC_HASH "unknown"
#endif
#ifndef SHINE_GIT_HEAD
#define SHINE_GIT_HEAD "unknown"
#endif

extern "C" const char* shine_build_id(void) { return "src " SHINE_SRC_HASH " git " SHINE_GIT_HEAD; }
