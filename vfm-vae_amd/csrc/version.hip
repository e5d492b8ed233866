// Library identification and kernel timing for the C ABI (include/vfmvae.h).
#include "vfm_common.h"

extern "C" const char* vfm_version(void) { return "vfmvae-hip 0.1.0 gfx950"; }

namespace vfm {
TimerArm& timer_arm() {
    static thread_local TimerArm t;
    return t;
}
int g_timer_mode = 1;
__global__ void timer_probe_kernel(int) {}
}  // namespace vfm

// Start-event binding of the kernel timer (see TimerArm): 1 = end of a probe kernel before the timed launch
// (default), 0 = the timed kernel's own dispatch. Returns the previous mode.
extern "C" int vfm_timer_mode(int mode) {
    const int prev = vfm::g_timer_mode;
    if (mode == 0 || mode == 1) vfm::g_timer_mode = mode;
    return prev;
}

// Arm (start, stop) for the following launches of this thread (both null: disarm). See TimerArm.
// Returns the number of launches made under the previous arming.
extern "C" int vfm_timer_arm(void* start, void* stop) {
    vfm::TimerArm& t = vfm::timer_arm();
    const int n = t.launches;
    t.start = (hipEvent_t)start;
    t.stop = (hipEvent_t)stop;
    t.launches = 0;
    t.first_only = false;
    return n;
}

// vfm_timer_arm for the first launch only: later launches of the call go untimed (see TimerArm).
extern "C" int vfm_timer_arm_first(void* start, void* stop) {
    const int n = vfm_timer_arm(start, stop);
    vfm::timer_arm().first_only = start != nullptr;
    return n;
}

// One empty one-wave kernel through VFM_LAUNCH (timed like any other launch when the timer is armed): the
// kernel timer's calibration of the fixed per-timed-launch interval (dispatch gap + an empty kernel).
extern "C" int vfm_timer_null_launch(void* stream) {
    VFM_LAUNCH(vfm::timer_probe_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, 0);
    return vfm::launch_status();
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
