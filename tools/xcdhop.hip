// xcdhop.hip — chained all-gather hops among 32 workgroups: every workgroup publishes one
// 128-B line of 16 granules {tag, value}, then gathers all 512 granules; the next hop starts
// when the gather is complete.  µs per hop for
//   LOCAL: the 32 workgroups of ONE XCD (membership from HW_REG_XCC_ID + an arrival counter),
//          plain stores (the line stays in that XCD's L2) + sc1 polls (L2-served);
//   SPREAD: blocks 0..31 (four per XCD under round-robin dealing), sc1 stores + sc1 polls.
// Poll variants (LOCAL): 8-byte loads (8 per lane) or 16-byte buffer loads (4 per lane), one or
// two poll rounds in flight, with or without draining the own publish first, with or without
// the other waves of the workgroup streaming LDS (the XCD kernel's off-critical dots).
//   hipcc --offload-arch=gfx950 -O3 tools/xcdhop.hip -o tools/xcdhop && tools/xcdhop
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kN = 32, kLine = 16;
typedef unsigned u4v __attribute__((ext_vector_type(4)));

__device__ inline unsigned xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 0xF; }

__device__ __forceinline__ u4v ld16(__amdgpu_buffer_rsrc_t r, int off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16 /* sc1 */);
}

template <bool LOCAL, int W16, int INFL, bool DRAIN, bool LDSLOAD>
__global__ __launch_bounds__(512) void hops(unsigned long long *vec, int *ctr, int nhops, unsigned long long *out) {
    __shared__ int s_idx;
    __shared__ float lds[8192];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) {
        int idx = -1;
        if (LOCAL) {
            if (xcc_id() == 0) idx = atomicAdd(ctr, 1);
        } else if (blockIdx.x < kN) {
            idx = blockIdx.x;
        }
        s_idx = idx < kN ? idx : -1;
    }
    for (int i = threadIdx.x; i < 8192; i += 512) lds[i] = (float)i;
    __syncthreads();
    const int me = s_idx;
    if (me < 0) return;
    if (wave != 0) {   // background: LDS streaming by the other waves (until wave 0 is done)
        if (!LDSLOAD) return;
        float acc = 0.0f;
        volatile int *flag = reinterpret_cast<volatile int *>(&s_idx);
        for (int it = 0; ; ++it) {
#pragma unroll 4
            for (int k = 0; k < 16; ++k) acc += lds[(lane * 4 + k * 256 + it) & 8191];
            if ((it & 63) == 0 && *flag < 0) break;
        }
        if (acc == 12345.0f) out[40] = 1;
        return;
    }
    const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + 200000000ull;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool dead = false;
    for (int h = 1; h <= nhops && !dead; ++h) {
        unsigned long long *v = vec + (size_t)(h & 1) * kN * kLine;
        if (lane < kLine) {
            const unsigned long long g = ((unsigned long long)h << 32) | (unsigned)(me * kLine + lane);
            if (LOCAL) __hip_atomic_store(v + me * kLine + lane, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            else __hip_atomic_store(v + me * kLine + lane, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (DRAIN) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (W16) {
            const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(v, 0, 0x7fffffff, 0x00020000);
            auto check = [&](const u4v (&x)[4]) {
                bool ok = true;
#pragma unroll
                for (int k = 0; k < 4; ++k) ok &= (x[k].y == (unsigned)h) & (x[k].w == (unsigned)h);
                return __all(ok);
            };
            u4v a[4], b[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) a[k] = ld16(r, 16 * (lane + 64 * k));
            if (INFL >= 3) {   // two poll rounds staggered by INFL shader cycles, kept staggered
                const unsigned long long s0 = __builtin_amdgcn_s_memtime();
                while (__builtin_amdgcn_s_memtime() - s0 < (unsigned long long)INFL) {
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) b[k] = ld16(r, 16 * (lane + 64 * k));
                for (;;) {
                    if (check(a)) break;
#pragma unroll
                    for (int k = 0; k < 4; ++k) a[k] = ld16(r, 16 * (lane + 64 * k));
                    if (check(b)) break;
#pragma unroll
                    for (int k = 0; k < 4; ++k) b[k] = ld16(r, 16 * (lane + 64 * k));
                    if (__builtin_amdgcn_s_memrealtime() > deadline) { dead = true; break; }
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                continue;
            }
            for (;;) {
                if (INFL == 2) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) b[k] = ld16(r, 16 * (lane + 64 * k));
                }
                if (check(a)) break;
                if (INFL == 2) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) a[k] = ld16(r, 16 * (lane + 64 * k));
                    if (check(b)) break;
                } else {
#pragma unroll
                    for (int k = 0; k < 4; ++k) a[k] = ld16(r, 16 * (lane + 64 * k));
                }
                if (__builtin_amdgcn_s_memrealtime() > deadline) { dead = true; break; }
            }
        } else {
            for (;;) {
                unsigned long long x[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) x[k] = __hip_atomic_load(v + lane + 64 * k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                bool ok = true;
#pragma unroll
                for (int k = 0; k < 8; ++k) ok &= (unsigned)(x[k] >> 32) == (unsigned)h;
                if (__all(ok)) break;
                if (__builtin_amdgcn_s_memrealtime() > deadline) { dead = true; break; }
            }
        }
    }
    if (lane == 0) {
        out[me] = dead ? ~0ull : __builtin_amdgcn_s_memrealtime() - t0;
        s_idx = -1;    // stop the background waves
    }
}

template <bool LOCAL, int W16, int INFL, bool DRAIN, bool LDSLOAD>
void run(unsigned long long *vec, int *ctr, unsigned long long *out, const char *name) {
    const int nhops = 20000;
    hipMemset(vec, 0, 2 * kN * kLine * 8 + 4096);
    hipMemset(ctr, 0, 4);
    hipMemset(out, 0, kN * 8);
    hipLaunchKernelGGL((hops<LOCAL, W16, INFL, DRAIN, LDSLOAD>), dim3(256), dim3(512), 0, 0, vec, ctr, nhops, out);
    hipDeviceSynchronize();
    unsigned long long h[kN];
    hipMemcpy(h, out, kN * 8, hipMemcpyDeviceToHost);
    unsigned long long mx = 0;
    bool dead = false;
    for (int i = 0; i < kN; ++i) {
        if (h[i] == ~0ull) dead = true;
        else if (h[i] > mx) mx = h[i];
    }
    printf("%-40s %s %.3f us per all-gather hop\n", name, dead ? "TIMEOUT" : "", mx * 10e-3 / nhops);
    fflush(stdout);
}


// Barrier-paced variant (the XCD kernel's Y hop): per hop, __syncthreads, then PUBW waves publish
// the workgroup's 16 granules (16 / PUBW each, by lanes 0.. of the wave), POLLW waves poll the
// whole vector (16-byte loads, 4 per lane), XPOLL: wave 7 also publishes + polls a second vector
// of the same shape (the h2 hand-off), then __syncthreads.
template <int PUBW, int POLLW, bool XPOLL, int NBAR = 2, int LS = kLine>
__global__ __launch_bounds__(512) void hops_paced(unsigned long long *vec, int *ctr, int nhops, unsigned long long *out) {
    __shared__ int s_idx;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) {
        int idx = -1;
        if (xcc_id() == 0) idx = atomicAdd(ctr, 1);
        s_idx = idx < kN ? idx : -1;
    }
    __syncthreads();
    const int me = s_idx;
    if (me < 0) return;
    const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + 200000000ull;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool dead = false;
    for (int h = 1; h <= nhops; ++h) {
        __syncthreads();
        unsigned long long *v = vec + (size_t)(h & 1) * kN * LS;
        unsigned long long *v2 = vec + 2 * kN * LS + (size_t)(h & 1) * kN * kLine;
        constexpr int per = kLine / PUBW;
        if (wave < PUBW && lane < per) {
            const int i = me * LS + wave * per + lane;
            __hip_atomic_store(v + i, ((unsigned long long)h << 32) | (unsigned)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (XPOLL && wave < PUBW && lane >= 32 && lane - 32 < per) {
            const int i = me * kLine + wave * per + lane - 32;
            __hip_atomic_store(v2 + i, ((unsigned long long)h << 32) | (unsigned)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        const bool poller = (wave >= 1 && wave <= POLLW) || (XPOLL && wave == 7);
        if (poller) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(wave == 7 ? v2 : v, 0, 0x7fffffff, 0x00020000);
            for (;;) {
                u4v a[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int gi = 2 * (lane + 64 * k), pi = wave == 7 ? gi : (gi / kLine) * LS + gi % kLine;
                    a[k] = ld16(r, 8 * pi);
                }
                bool ok = true;
#pragma unroll
                for (int k = 0; k < 4; ++k) ok &= (a[k].y == (unsigned)h) & (a[k].w == (unsigned)h);
                if (__all(ok)) break;
                if (__builtin_amdgcn_s_memrealtime() > deadline) { dead = true; break; }
            }
        }
        if (NBAR == 2) {
            if (__syncthreads_or(dead)) break;
        } else if (NBAR == 3) {
            __syncthreads();
            if (dead) break;
        } else if (dead) {
            break;
        }
    }
    if (threadIdx.x == 64) out[me] = dead ? ~0ull : __builtin_amdgcn_s_memrealtime() - t0;
}

template <int PUBW, int POLLW, bool XPOLL, int NBAR = 2, int LS = kLine>
void run_paced(unsigned long long *vec, int *ctr, unsigned long long *out, const char *name) {
    const int nhops = 20000;
    hipMemset(vec, 0, 1 << 20);
    hipMemset(ctr, 0, 4);
    hipMemset(out, 0, kN * 8);
    hipLaunchKernelGGL((hops_paced<PUBW, POLLW, XPOLL, NBAR, LS>), dim3(256), dim3(512), 0, 0, vec, ctr, nhops, out);
    hipDeviceSynchronize();
    unsigned long long h[kN];
    hipMemcpy(h, out, kN * 8, hipMemcpyDeviceToHost);
    unsigned long long mx = 0;
    bool dead = false;
    for (int i = 0; i < kN; ++i) {
        if (h[i] == ~0ull) dead = true;
        else if (h[i] > mx) mx = h[i];
    }
    printf("%-40s %s %.3f us per paced hop\n", name, dead ? "TIMEOUT" : "", mx * 10e-3 / nhops);
    fflush(stdout);
}

// Poll round trip: wave 0 of 32 workgroups of one XCD polls a vector that never completes,
// NR rounds of 4 x 16-byte sc1 loads (each round waits for the previous one)
__global__ __launch_bounds__(512) void poll_rtt(unsigned long long *vec, int *ctr, unsigned long long *out) {
    __shared__ int s_idx;
    if (threadIdx.x == 0) {
        int idx = -1;
        if (xcc_id() == 0) idx = atomicAdd(ctr, 1);
        s_idx = idx < kN ? idx : -1;
    }
    __syncthreads();
    const int me = s_idx, lane = threadIdx.x & 63;
    if (me < 0 || threadIdx.x >= 64) return;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(vec, 0, 0x7fffffff, 0x00020000);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned acc = 0;
    for (int it = 0; it < 20000; ++it) {
        asm volatile("" ::: "memory");   // keep the loads in the loop
        u4v a[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) a[k] = ld16(r, 16 * (lane + 64 * k));
#pragma unroll
        for (int k = 0; k < 4; ++k) acc += a[k].y + a[k].w;
        if (__all(acc == 0xFFFFFFFFu)) break;
    }
    if (lane == 0) out[me] = __builtin_amdgcn_s_memrealtime() - t0 + (acc == 1234567u);
}

int main() {
    unsigned long long *vec, *out;
    int *ctr;
    hipMalloc(&vec, 1 << 20);   // ≥ 8192 granules + slack
    hipMalloc(&out, 64 * 8);
    hipMalloc(&ctr, 64);
    {
        hipMemset(vec, 0, 1 << 20);
        hipMemset(ctr, 0, 4);
        hipLaunchKernelGGL(poll_rtt, dim3(256), dim3(512), 0, 0, vec, ctr, out);
        hipDeviceSynchronize();
        unsigned long long h[kN], mx = 0;
        hipMemcpy(h, out, kN * 8, hipMemcpyDeviceToHost);
        for (int i = 0; i < kN; ++i) mx = h[i] > mx ? h[i] : mx;
        printf("%-40s %.3f us per poll round\n", "LOCAL 16B x4 poll round trip", mx * 10e-3 / 20000);
    }
    for (int r = 0; r < 1; ++r) {
        run<true, 0, 1, false, false>(vec, ctr, out, "LOCAL 8B x8");
        run<true, 0, 1, true, false>(vec, ctr, out, "LOCAL 8B x8 drain");
        run<true, 1, 1, false, false>(vec, ctr, out, "LOCAL 16B x4");
        run<true, 1, 1, true, false>(vec, ctr, out, "LOCAL 16B x4 drain");
        run<true, 1, 2, true, false>(vec, ctr, out, "LOCAL 16B x4 drain, 2 rounds in flight");
        run<true, 1, 150, true, false>(vec, ctr, out, "LOCAL 16B x4 drain, 2 rounds stagger 150");
        run<true, 1, 300, true, false>(vec, ctr, out, "LOCAL 16B x4 drain, 2 rounds stagger 300");
        run<true, 1, 450, true, false>(vec, ctr, out, "LOCAL 16B x4 drain, 2 rounds stagger 450");
        run<true, 1, 600, true, false>(vec, ctr, out, "LOCAL 16B x4 drain, 2 rounds stagger 600");
        run<true, 1, 1, true, true>(vec, ctr, out, "LOCAL 16B x4 drain, LDS-streaming waves");
        run<false, 0, 1, false, false>(vec, ctr, out, "SPREAD 8B x8 (sc1 stores)");
        run_paced<1, 1, false, 1>(vec, ctr, out, "PACED 1 pub, 1 poller, one plain barrier");
        run_paced<1, 1, false, 3>(vec, ctr, out, "PACED 1 pub, 1 poller, two barriers");
        run_paced<8, 1, false, 3>(vec, ctr, out, "PACED 8 publisher waves, 1 poller");
        run_paced<1, 2, false, 3>(vec, ctr, out, "PACED 1 publisher wave, 2 pollers");
        run_paced<8, 2, false, 3>(vec, ctr, out, "PACED 8 publisher waves, 2 pollers");
        run_paced<8, 1, true, 3>(vec, ctr, out, "PACED 8 pub, 1 poller + h2 vector poller");
        run_paced<8, 2, true, 3>(vec, ctr, out, "PACED 8 pub, 2 pollers + h2 vector poller");
        run_paced<8, 1, false, 3, 32>(vec, ctr, out, "PACED 8 pub, 1 poller, lines 256 B apart");
        run_paced<8, 1, false, 3, 128>(vec, ctr, out, "PACED 8 pub, 1 poller, lines 1 KiB apart");
        run_paced<8, 1, false, 3, 512>(vec, ctr, out, "PACED 8 pub, 1 poller, lines 4 KiB apart");
        run_paced<1, 1, false, 3, 128>(vec, ctr, out, "PACED 1 pub, 1 poller, lines 1 KiB apart");
        run_paced<8, 1, false, 3>(vec, ctr, out, "PACED 8 publisher waves, 1 poller (again)");
    }
    return 0;
}
