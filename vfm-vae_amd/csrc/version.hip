// Library identification for the C ABI (include/vfmvae.h).
#include "vfm_common.h"

extern "C" const char* vfm_version(void) { return "vfmvae-hip 0.1.0 gfx950"; }
