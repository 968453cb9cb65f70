// xcdhop.hip — chained all-gather hops among 32 workgroups: every workgroup publishes one
// 128-B line of 16 granules {tag, value}, then gathers all 512 granules; the next hop starts
// when the gather is complete.  µs per hop for
//   LOCAL: the 32 workgroups of ONE XCD (membership from HW_REG_XCC_ID + an arrival counter),
//          plain stores (the line stays in that XCD's L2) + sc1 polls (L2-served);
//   SPREAD: blocks 0..31 (four per XCD under round-robin dealing), sc1 stores + sc1 polls.
//   hipcc --offload-arch=gfx950 -O3 tools/xcdhop.hip -o tools/xcdhop && tools/xcdhop
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kN = 32, kLine = 16;

__device__ inline unsigned xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 0xF; }

template <bool LOCAL>
__global__ __launch_bounds__(256) void hops(unsigned long long *vec, int *ctr, int nhops, unsigned long long *out) {
    __shared__ int s_idx;
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
    __syncthreads();
    const int me = s_idx;
    if (me < 0 || wave != 0) return;
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
    if (lane == 0) {
        out[me] = dead ? ~0ull : __builtin_amdgcn_s_memrealtime() - t0;
    }
}

template <bool LOCAL>
void run(unsigned long long *vec, int *ctr, unsigned long long *out) {
    const int nhops = 20000;
    hipMemset(vec, 0, 2 * kN * kLine * 8 + 4096);
    hipMemset(ctr, 0, 4);
    hipMemset(out, 0, kN * 8);
    hipLaunchKernelGGL((hops<LOCAL>), dim3(256), dim3(256), 0, 0, vec, ctr, nhops, out);
    hipDeviceSynchronize();
    unsigned long long h[kN];
    int c = 0;
    hipMemcpy(h, out, kN * 8, hipMemcpyDeviceToHost);
    hipMemcpy(&c, ctr, 4, hipMemcpyDeviceToHost);
    unsigned long long mx = 0;
    bool dead = false;
    for (int i = 0; i < kN; ++i) {
        if (h[i] == ~0ull) dead = true;
        else if (h[i] > mx) mx = h[i];
    }
    printf("%-6s (xcc0 arrivals %d): %s %.3f us per all-gather hop\n", LOCAL ? "LOCAL" : "SPREAD", c,
           dead ? "TIMEOUT" : "", mx * 10e-3 / nhops);
    fflush(stdout);
}

int main() {
    unsigned long long *vec, *out;
    int *ctr;
    hipMalloc(&vec, 1 << 20);
    hipMalloc(&out, kN * 8);
    hipMalloc(&ctr, 64);
    for (int r = 0; r < 2; ++r) {
        run<true>(vec, ctr, out);
        run<false>(vec, ctr, out);
    }
    return 0;
}
