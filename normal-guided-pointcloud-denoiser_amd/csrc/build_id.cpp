// libpcd's build id: a hash of every source file the library is compiled from plus the extra compile flags (the
// Makefile computes it), so a profile or traffic file can name the build it measured and the bench can tell when
// its counters come from another build.
#include "pcd.h"

#ifndef PCD_BUILD_ID
#define PCD_BUILD_ID "unknown"
#endif

extern "C" const char* pcd_build_id(void) { return PCD_BUILD_ID; }
