// mfma_poll.hip — does a wave's MFMA stream delay the vector-memory load that follows it?
//
// Round-6 diagnostic for DESIGN.md §4.3a: in the deepmind kernel a hop poll issued by a wave right
// after its R·h MFMA stream ended ≈ 0.4 µs after the data were visible to an idle wave.  Here one
// workgroup per CU (4 waves, one per SIMD) times, on wave `w`, the latency of one 16-byte sc1 load
// of an L2-resident line issued (mode 0) after n back-to-back v_mfma_f32_4x4x1_16b_f32, (mode 1)
// before them and consumed after, (mode 2) after them and an s_sleep, (mode 3) after n dependent
// VALU FMAs instead.  The other waves run the same stream (like a layer) or idle (flag).
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_poll.hip -o tools/mfma_poll && tools/mfma_poll
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f4v __attribute__((ext_vector_type(4)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u4v ld16_sc1(__amdgpu_buffer_rsrc_t r, int off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16 /* sc1 */);
}

template <int kMode, int n>
__global__ __launch_bounds__(256, 1) void probe(const unsigned *line, unsigned long long *out, int others) {
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned *>(line), 0, 0x7fffffff,
                                                                        0x00020000);
    const int off = ((blockIdx.x * 64 + lane) & 1023) * 16;
    // warm the line into L2 (and wait)
    u4v w = ld16_sc1(r, off);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    float a = (float)lane * 1e-3f + (float)w.x * 1e-30f, b = 1.0f;
    f4v acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
    const bool probe_wave = wave == 1;
    const bool run = probe_wave || others;
    unsigned long long t0 = 0, t1 = 0, t2 = 0;
    u4v v = {0, 0, 0, 0};
    if (run) {
        t0 = __builtin_amdgcn_s_memtime();
        if (kMode == 1 && probe_wave) v = ld16_sc1(r, off);
        if (kMode == 3) {
            float x = a;
#pragma unroll
            for (int i = 0; i < n; ++i) x = __builtin_fmaf(x, 1.0001f, b);
            acc[0].x = x;
        } else {
#pragma unroll
            for (int i = 0; i < n; ++i) acc[i & 3] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[i & 3], 0, 0, 0);
        }
        if (kMode == 2 && probe_wave) __builtin_amdgcn_s_sleep(8);
        t1 = __builtin_amdgcn_s_memtime();
        if (kMode != 1 && probe_wave) v = ld16_sc1(r, off);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        t2 = __builtin_amdgcn_s_memtime();
    }
    const float s = (acc[0].x + acc[1].y) + (acc[2].z + acc[3].w) + (float)v.y * 1e-30f;
    if (probe_wave && lane == 0) {
        out[blockIdx.x * 3 + 0] = t1 - t0;
        out[blockIdx.x * 3 + 1] = t2 - t1;
        out[blockIdx.x * 3 + 2] = __float_as_uint(s);
    }
}

int main() {
    const int G = 256;
    unsigned *line;
    unsigned long long *out;
    hipMalloc(&line, 1024 * 16);
    hipMemset(line, 0, 1024 * 16);
    hipMalloc(&out, G * 3 * 8);
    std::vector<unsigned long long> h(G * 3);
    const char *names[] = {"load after MFMAs", "load before MFMAs, waited after", "load after MFMAs + s_sleep 8",
                           "load after dependent FMAs"};
    auto launch = [&](int mode, int n, int others) {
#define WRNN_P(M, N) if (mode == M && n == N) hipLaunchKernelGGL((probe<M, N>), dim3(G), dim3(256), 0, 0, line, out, others);
#define WRNN_PN(M) WRNN_P(M, 0) WRNN_P(M, 16) WRNN_P(M, 64) WRNN_P(M, 128) WRNN_P(M, 256)
        WRNN_PN(0) WRNN_PN(1) WRNN_PN(2) WRNN_PN(3)
    };
    for (int mode = 0; mode < 4; ++mode)
        for (int others = 0; others < 2; ++others)
            for (int n : {0, 16, 64, 128, 256}) {
                for (int rep = 0; rep < 2; ++rep) {
                    launch(mode, n, others);
                    hipDeviceSynchronize();
                }
                hipMemcpy(h.data(), out, G * 3 * 8, hipMemcpyDeviceToHost);
                std::vector<unsigned long long> a, b;
                for (int g = 0; g < G; ++g) {
                    a.push_back(h[g * 3]);
                    b.push_back(h[g * 3 + 1]);
                }
                std::sort(a.begin(), a.end());
                std::sort(b.begin(), b.end());
                printf("%-34s others %d n %3d: stream %6llu cyc, load %5llu cyc (median over %d CUs; p90 %llu)\n",
                       names[mode], others, n, a[G / 2], b[G / 2], G, b[G * 9 / 10]);
            }
    return 0;
}
