// rows_device.h — device helpers of the multi-row kernels (fatchord_rows.hip, deepmind_rows.hip):
// per-producer flag polls and sc1 stores of the bulk hand-offs.
#pragma once
#include "fatchord_rows.h"
#include "wrnn_device.h"

namespace wrnn {

// One wave waits until every producer flag of a hop holds >= want (flags are monotonic).
// kFlagSlots = 256 slots are always allocated, so the four unconditional loads stay in bounds.
__device__ __forceinline__ void wait_flags(const unsigned *f, int n, unsigned want, int *ctl, long long timeout,
                                           int step, int hop, int *lds_abort) {
    const int lane = threadIdx.x & 63;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned spins = 0;
    for (;;) {
        unsigned v[kFlagSlots / 64];
#pragma unroll
        for (int k = 0; k < kFlagSlots / 64; ++k)
            v[k] = __hip_atomic_load(f + (lane + 64 * k) * kFlagStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool ok = true;
#pragma unroll
        for (int k = 0; k < kFlagSlots / 64; ++k) ok &= (lane + 64 * k >= n) | (v[k] >= want);
        if (ok) break;
        if ((++spins & 63u) == 0) {
            const bool late = (long long)(__builtin_amdgcn_s_memrealtime() - t0) > timeout;
            const bool other = __hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
            if (late || other) {
                if (late) record_abort(ctl, -4, step, hop, blockIdx.x);
                *lds_abort = 1;
                break;
            }
        }
    }
}

__device__ __forceinline__ void store_sc1(float *p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace wrnn
