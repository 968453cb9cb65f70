// xcdbench.hip — one-way hand-off latency between two workgroups on the SAME XCD vs on
// DIFFERENT XCDs, for store flavours that keep the line in the producer XCD's L2 (plain,
// workgroup-scope) or write it through (agent sc1).  The consumer always polls with agent-scope
// relaxed loads (sc1: bypass L1, served by L2 / beyond).  Blocks are dealt round-robin over the
// 8 XCDs, so blocks 0 and 8 share one; the XCC id is read back from the hardware register.
//   hipcc --offload-arch=gfx950 -O3 tools/xcdbench.hip -o tools/xcdbench && tools/xcdbench
#include <hip/hip_runtime.h>

#include <cstdio>

enum St { ST_AGENT, ST_WG, ST_PLAIN };
static const char *stn[] = {"store rlx agent (sc1)", "store rlx workgroup", "store rlx singlethread"};

__device__ inline unsigned xcc_id() {
    // HW_REG_XCC_ID (id 20), bits [3:0]
    return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 0xF;
}

template <int ST>
__device__ inline void put(unsigned long long *p, unsigned long long v) {
    if (ST == ST_AGENT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if (ST == ST_WG) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SINGLETHREAD);
}

// blocks a and b ping-pong `rounds` times; every other block exits at once
template <int ST>
__global__ void pp(unsigned long long *w, int rounds, unsigned long long *out, int a, int b) {
    const int me = blockIdx.x;
    if (threadIdx.x != 0 || (me != a && me != b)) return;
    const int side = me == a ? 0 : 1;
    unsigned long long *mine = w + side * 64, *theirs = w + (1 - side) * 64;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long c0 = __builtin_amdgcn_s_memrealtime() + 200000000ull;   // 2 s bound
    for (int r = 1; r <= rounds; ++r) {
        if (side == 1 || r > 1) {
            const unsigned long long want = side == 1 ? r : r - 1;
            for (;;) {
                const unsigned long long v = __hip_atomic_load(theirs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (v >= want) break;
                if (__builtin_amdgcn_s_memrealtime() > c0) {
                    out[4 + side] = 1;   // timed out
                    r = rounds + 1;
                    break;
                }
            }
        }
        put<ST>(mine, (unsigned long long)r);
    }
    out[side] = __builtin_amdgcn_s_memrealtime() - t0;
    out[2 + side] = xcc_id();
}

template <int ST>
void run(unsigned long long *w, unsigned long long *out, int a, int b) {
    const int rounds = 4000;
    hipMemset(w, 0, 1 << 16);
    hipMemset(out, 0, 64);
    hipLaunchKernelGGL((pp<ST>), dim3(16), dim3(64), 0, 0, w, rounds, out, a, b);
    hipDeviceSynchronize();
    unsigned long long h[6];
    hipMemcpy(h, out, 48, hipMemcpyDeviceToHost);
    const double us = (h[0] > h[1] ? h[0] : h[1]) * 10e-3 / rounds / 2;
    printf("%-22s blocks %2d,%2d (xcc %llu,%llu)%s: %.3f us one-way\n", stn[ST], a, b, h[2], h[3],
           (h[4] || h[5]) ? " TIMEOUT" : "", us);
    fflush(stdout);
}

int main() {
    unsigned long long *w, *out;
    hipMalloc(&w, 1 << 16);
    hipMalloc(&out, 64);
    for (int rep = 0; rep < 2; ++rep) {
        run<ST_AGENT>(w, out, 0, 8);
        run<ST_AGENT>(w, out, 0, 1);
        run<ST_WG>(w, out, 0, 8);
        run<ST_WG>(w, out, 0, 1);
        run<ST_PLAIN>(w, out, 0, 8);
        run<ST_PLAIN>(w, out, 0, 1);
    }
    return 0;
}
