// otf_common.hip — library identification and host helpers.
#include <mutex>

#include "otf_device.h"

namespace otf {

int check_hip(hipError_t e) {
    (void)hipGetLastError();  // clear the sticky per-thread error for the next call
    return e == hipSuccess ? OTF_OK : OTF_EHIP;
}

int device_cu_count() {
    static std::mutex mu;
    static int cache[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    std::lock_guard<std::mutex> lk(mu);
    if (cache[dev] == 0) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            cus <= 0)
            cus = 256;
        cache[dev] = cus;
    }
    return cache[dev];
}

}  // namespace otf

extern "C" const char* otf_version(void) { return "otfuse 0.1.0 gfx950"; }
