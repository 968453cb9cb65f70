// pollbench.hip — measure the round trip of one polling pass (agent-scope sc1 loads of
// 8-byte granules) as a function of how many workgroups poll, how many replicas the polled
// vector has and how far apart the replicas sit.  Each workgroup: 2 polling waves, each lane
// keeps `per_lane` loads in flight per pass; 'passes' passes, timed with s_memrealtime.
//   hipcc --offload-arch=gfx950 -O3 tools/pollbench.hip -o pollbench && ./pollbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void poll_kernel(const unsigned long long *buf, int reps, long long rep_stride,
                                                   int per_lane, int passes, unsigned long long *out) {
    const int tid = threadIdx.x;
    if (tid >= 128) return;
    const unsigned long long *g = buf + (size_t)(blockIdx.x % reps) * rep_stride;
    unsigned long long acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int p = 0; p < passes; ++p) {
        unsigned long long v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (k < per_lane) v[k] = __hip_atomic_load(g + tid + k * 128, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (k < per_lane) acc += v[k];
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) out[blockIdx.x * 2] = t1 - t0;
    if (acc == 12345) out[blockIdx.x * 2 + 1] = acc;
}

int main() {
    const size_t bytes = 64ull << 20;
    unsigned long long *buf, *out;
    hipMalloc(&buf, bytes);
    hipMemset(buf, 0, bytes);
    hipMalloc(&out, 256 * 2 * 8);
    const int passes = 200;
    std::vector<unsigned long long> h(512);
    printf("%6s %5s %10s %8s %12s\n", "grid", "reps", "stride_B", "per_lane", "us/pass");
    for (int grid : {32, 64, 128, 256})
        for (int reps : {1, 8, 32})
            for (long long stride_b : {4096LL, 4352LL, 65536LL})
                for (int per_lane : {4, 8}) {
                    if (reps == 1 && stride_b != 4096) continue;
                    hipLaunchKernelGGL(poll_kernel, dim3(grid), dim3(256), 0, 0, buf, reps, stride_b / 8, per_lane, 10, out);
                    hipLaunchKernelGGL(poll_kernel, dim3(grid), dim3(256), 0, 0, buf, reps, stride_b / 8, per_lane, passes, out);
                    hipDeviceSynchronize();
                    hipMemcpy(h.data(), out, grid * 2 * 8, hipMemcpyDeviceToHost);
                    double mx = 0, sum = 0;
                    for (int i = 0; i < grid; ++i) { double v = h[2 * i] * 10e-3 / passes; sum += v; mx = v > mx ? v : mx; }
                    printf("%6d %5d %10lld %8d %8.3f avg %6.3f max\n", grid, reps, stride_b, per_lane, sum / grid, mx);
                }
    return 0;
}
