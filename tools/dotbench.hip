// dotbench.hip — cost of one round of the rows kernel's blocked dot engines in isolation:
// one workgroup of 4 waves (16 engines), weights and a tile of activation rows in LDS, each
// engine runs bdot4<NW, KI> `reps` times.  Prints ns per round.
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -I../wavernn_amd/csrc tools/dotbench.hip -o tools/dotbench
#include <hip/hip_runtime.h>

#include <cstdio>

#include "wrnn_device.h"

using namespace wrnn;

template <int NW, int KI, int WAVES>
__global__ __launch_bounds__(256) void bench(const float *g, float *sink, int reps, unsigned long long *cyc) {
    __shared__ __attribute__((aligned(16))) float lds[16 * 512 + 8 * 512];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, row = lane >> 4;
    for (int i = tid; i < 16 * 512 + 8 * 512; i += 256) lds[i] = g[i];
    __syncthreads();
    const float *W = lds, *X = lds + 16 * 512;
    float s = 0.0f;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (wave < WAVES)
        for (int r = 0; r < reps; ++r) {
            float acc[NW];
            const int e = wave * 4 + row;
            bdot4<NW, KI>(W + (e % 4) * NW * 512, 512, X + (e / 4) * 4 * 512 % (4 * 512), 512, 4, 128, li, acc);
#pragma unroll
            for (int i = 0; i < NW; ++i) s += acc[i];
            asm volatile("" ::: "memory");
        }
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) cyc[0] = t1 - t0;
    sink[tid] = s;
}

template <int NW, int KI, int WAVES>
void run(const float *g, float *sink, unsigned long long *cyc) {
    const int reps = 1000;
    hipLaunchKernelGGL((bench<NW, KI, WAVES>), dim3(1), dim3(256), 0, 0, g, sink, reps, cyc);
    hipDeviceSynchronize();
    unsigned long long c = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("bdot4<%d,%d> waves=%d: %.1f ns per round (%d FMA/lane)\n", NW, KI, WAVES, c * 10.0 / reps, NW * 4 * 4 * KI);
    fflush(stdout);
}

int main() {
    float *g, *sink;
    unsigned long long *cyc;
    hipMalloc(&g, 24 * 512 * 4);
    hipMalloc(&sink, 256 * 4);
    hipMalloc(&cyc, 8);
    hipMemset(g, 0, 24 * 512 * 4);
    run<3, 8, 4>(g, sink, cyc);
    run<3, 8, 1>(g, sink, cyc);
    run<2, 8, 4>(g, sink, cyc);
    run<3, 0, 4>(g, sink, cyc);
    run<1, 8, 4>(g, sink, cyc);
    return 0;
}
