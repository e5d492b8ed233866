// Library identification and kernel timing for the C ABI (include/vfmvae.h).
#include "vfm_common.h"

extern "C" const char* vfm_version(void) { return "vfmvae-hip 0.1.0 gfx950"; }

namespace vfm {
TimerArm& timer_arm() {
    static thread_local TimerArm t;
    return t;
}
}  // namespace vfm

// Arm (start, stop) for the following launches of this thread (both null: disarm). See TimerArm.
// Returns the number of launches made under the previous arming.
extern "C" int vfm_timer_arm(void* start, void* stop) {
    vfm::TimerArm& t = vfm::timer_arm();
    const int n = t.launches;
    t.start = (hipEvent_t)start;
    t.stop = (hipEvent_t)stop;
    t.launches = 0;
    return n;
}

extern "C" int vfm_event_create(void** ev) {
    if (!ev) return VFM_ERR_ARGS;
    hipEvent_t e = nullptr;
    const hipError_t r = hipEventCreate(&e);
    *ev = (void*)e;
    return r == hipSuccess ? VFM_OK : (int)r;
}

extern "C" int vfm_event_destroy(void* ev) {
    return ev && hipEventDestroy((hipEvent_t)ev) == hipSuccess ? VFM_OK : VFM_ERR_ARGS;
}

// Milliseconds between two completed events (synchronises on `stop`).
extern "C" int vfm_event_elapsed(void* start, void* stop, float* ms) {
    if (!start || !stop || !ms) return VFM_ERR_ARGS;
    hipError_t r = hipEventSynchronize((hipEvent_t)stop);
    if (r != hipSuccess) return (int)r;
    r = hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop);
    return r == hipSuccess ? VFM_OK : (int)r;
}
