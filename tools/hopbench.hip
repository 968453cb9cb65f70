// hopbench.hip — an isolated all-gather hand-off, the unit the WaveRNN loop repeats 4-5×
// per sample: every workgroup publishes its `per_wg` values as 8-byte {tag, value} granules
// (agent-scope sc1 stores, to every replica), then polls the whole vector (one replica) until
// every tag equals the round, then the next round starts.  µs per round = one hop.
// Variants: replicas, granule padding (values of one producer share a line vs own line),
// polling waves, and whether the poll loop sleeps.
//   hipcc --offload-arch=gfx950 -O3 tools/hopbench.hip -o hopbench && ./hopbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

struct Cfg {
    int reps;        // replicas of the vector
    int pad;         // granule slots per producer (>= per_wg); 8 = one 64-B line per producer
    int poll_waves;  // waves that poll (each lane polls N/(64*poll_waves) granules)
    int sleep;       // s_sleep between passes
};

__device__ __forceinline__ void store16_sc1(unsigned long long *p, unsigned long long a, unsigned long long b) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4 v = {(unsigned)a, (unsigned)(a >> 32), (unsigned)b, (unsigned)(b >> 32)};
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

// v4: the poll pass issues NG unconditional loads (addresses clamped into range), then checks
// them: one memory round trip per pass instead of one per guarded load.
template <int NG>
__global__ __launch_bounds__(256) void hop_kernel_v3(unsigned long long *buf, long long rep_stride, int per_wg, int pad,
                                                     int reps, int rounds, unsigned long long *out, int full, int delay,
                                                     int pollers) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int G = gridDim.x, N = G * per_wg;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int r = 0; r < rounds; ++r) {
        const unsigned tag = r + 1;
        if (wave == 3) {
            if (lane < reps)
                for (int u = 0; u < per_wg; ++u)
                    __hip_atomic_store(buf + lane * rep_stride + (size_t)blockIdx.x * pad + u,
                                       ((unsigned long long)tag << 32) | u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (wave < pollers) {
            const unsigned long long *g = buf + (size_t)(blockIdx.x % reps) * rep_stride;
            const int np = 64 * pollers;
            const unsigned long long *addr[NG];
#pragma unroll
            for (int k = 0; k < NG; ++k) {
                int i = tid + k * np;
                i = i < N ? i : (tid < N ? tid : 0);
                addr[k] = g + (size_t)(i / per_wg) * pad + (i % per_wg);
            }
            for (;;) {
                unsigned long long v[NG];
#pragma unroll
                for (int k = 0; k < NG; ++k) v[k] = __hip_atomic_load(addr[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                bool ok = true;
#pragma unroll
                for (int k = 0; k < NG; ++k) ok &= (unsigned)(v[k] >> 32) >= tag;
                if (ok) break;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) out[blockIdx.x] = t1 - t0;
}

template <int SLEEP>
__global__ __launch_bounds__(256) void hop_kernel(unsigned long long *buf, long long rep_stride, int per_wg,
                                                  int pad, int reps, int poll_waves, int rounds,
                                                  unsigned long long *out, int full) {
    __shared__ int done_flag;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int G = gridDim.x, N = G * per_wg;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int r = 0; r < rounds; ++r) {
        const unsigned tag = r + 1;
        if (full && wave == 3) {
            // every producer writes its whole padded slot (pad granules) with 16-B sc1 stores
            const int lanes_per_rep = pad / 2;
            const int rep = lane / lanes_per_rep, q = lane % lanes_per_rep;
            if (rep < reps && lanes_per_rep * reps <= 64) {
                const unsigned long long x = ((unsigned long long)tag << 32);
                store16_sc1(buf + rep * rep_stride + (size_t)blockIdx.x * pad + 2 * q, x | (2 * q), x | (2 * q + 1));
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if (wave == 3 && lane < reps) {
            for (int u = 0; u < per_wg; ++u) {
                const unsigned long long x = ((unsigned long long)tag << 32) | (unsigned)(blockIdx.x * per_wg + u);
                __hip_atomic_store(buf + lane * rep_stride + (size_t)blockIdx.x * pad + u, x, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (wave < poll_waves) {
            const unsigned long long *g = buf + (size_t)(blockIdx.x % reps) * rep_stride;
            const int np = 64 * poll_waves;
            const int mine = (N + np - 1) / np;
            unsigned long long v[16];
            unsigned done = 0, all = (1u << mine) - 1;
            while (done != all) {
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const int i = tid + k * np;
                    if (k < mine && !(done & (1u << k)) && i < N)
                        v[k] = __hip_atomic_load(g + (size_t)(i / per_wg) * pad + (i % per_wg), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
                }
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const int i = tid + k * np;
                    if (k < mine && !(done & (1u << k)) && (i >= N || (unsigned)(v[k] >> 32) >= tag)) done |= 1u << k;   // >=: a fast producer may already be a round ahead
                }
                if (SLEEP && done != all) __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) out[blockIdx.x] = t1 - t0;
    (void)done_flag;
}

int main() {
    unsigned long long *buf, *out;
    const size_t bytes = 64ull << 20;
    hipMalloc(&buf, bytes);
    hipMalloc(&out, 256 * 8);
    std::vector<unsigned long long> h(256);
    const int rounds = 1000;
    printf("%5s %5s %4s %4s %6s %10s\n", "grid", "perwg", "pad", "reps", "pollw", "us/hop");
    for (int reps : {1, 8})
        for (int pad : {0, 8})
            for (int grid : {2, 8, 32, 64, 128, 256}) {
                const int per_wg = grid == 256 ? 2 : (grid >= 64 ? 512 / grid : 2);
                const int padv = pad ? (pad > per_wg ? pad : per_wg) : per_wg;
                const int N = grid * per_wg;
                for (int pw : {1, 2}) {
                    const int ng = (N + 64 * pw - 1) / (64 * pw);
                    const long long stride = ((long long)grid * padv * 8 + 65535) / 65536 * 65536 / 8;
                    hipMemset(buf, 0, bytes);
                    auto k = ng <= 1 ? hop_kernel_v3<1> : ng <= 2 ? hop_kernel_v3<2> : ng <= 4 ? hop_kernel_v3<4> : hop_kernel_v3<8>;
                    hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, buf, stride, per_wg, padv, reps, rounds, out, 0, 0, pw);
                    hipDeviceSynchronize();
                    hipMemcpy(h.data(), out, grid * 8, hipMemcpyDeviceToHost);
                    double mx = 0;
                    for (int i = 0; i < grid; ++i) mx = h[i] > mx ? h[i] : mx;
                    printf("%5d %5d %4d %4d %6d %10.3f\n", grid, per_wg, padv, reps, pw, mx * 10e-3 / rounds);
                    fflush(stdout);
                }
            }
    return 0;
}
