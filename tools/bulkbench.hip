// bulkbench.hip — per-round cost of the bulk hand-off a multi-row step needs: every workgroup
// publishes its 2 values for each of B rows (sc1 stores), drains its stores, then signals; every
// workgroup waits for all signals and loads the whole [B][512] matrix (sc1 loads) into LDS.
// Signalling: SIG 0 = replicated counter (8 replicas, agent atomic add by 8 lanes; consumer
// polls replica w % 8); SIG 1 = one flag per producer (consumer polls all G flags).
//   hipcc --offload-arch=gfx950 -O3 tools/bulkbench.hip -o tools/bulkbench && tools/bulkbench
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int R = 512, U = 2, kThreads = 256, kReps = 8, kRepStride = 64;   // counter replicas 512 B apart

template <int SIG, int LD, int V>
__global__ __launch_bounds__(kThreads) void bulk(float *buf, unsigned *ctr, unsigned *flags, int B, int rounds,
                                                 unsigned long long *out, float *sink) {
    extern __shared__ float act[];                    // [B][R]
    const int w = blockIdx.x, G = gridDim.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    float acc = 0.0f;
    for (int r = 0; r < rounds; ++r) {
        float *cur = buf + (size_t)(LD == 2 ? r : (r & 1)) * B * R;
        // publish: B rows × U values of this workgroup (wave 1)
        if (wave == 1)
            for (int i = lane; i < B * U; i += 64) {
                const int b = i / U, u = i - b * U;
                __hip_atomic_store(cur + b * R + w * U + u, (float)(r + b + u + acc * 0.0f), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        if (wave == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (wave == 1) {
            if (SIG == 0) {
                if (lane < kReps)
                    __hip_atomic_fetch_add(ctr + lane * kRepStride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else if (lane == 0) {
                __hip_atomic_store(flags + w * 16, (unsigned)(r + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        // wait (wave 0)
        if (wave == 0) {
            if (SIG == 0) {
                const unsigned want = (unsigned)G * (r + 1);
                if (lane == 0)
                    while (__hip_atomic_load(ctr + (w % kReps) * kRepStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {}
            } else {
                for (;;) {
                    bool ok = true;
                    for (int p = lane; p < G; p += 64)
                        ok &= __hip_atomic_load(flags + p * 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)(r + 1);
                    if (__all(ok)) break;
                }
            }
        }
        __syncthreads();
        // bulk load [B][R] into LDS: LD 0 = 16-B sc1 buffer loads to registers then ds_write,
        // LD 1 = 16-B sc1 LDS-DMA (global_load_lds_dwordx4 sc1)
        if (LD == 0) {
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(cur, 0, B * R * 4, 0x00020000);
            constexpr int kU = 4;
            for (int i0 = tid; i0 < B * R / 4; i0 += kThreads * kU) {
                float4 v[kU];
#pragma unroll
                for (int k = 0; k < kU; ++k) {
                    const int i = i0 + k * kThreads;
                    v[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, (i < B * R / 4 ? i : 0) * 16, 0, 16));
                }
#pragma unroll
                for (int k = 0; k < kU; ++k) {
                    const int i = i0 + k * kThreads;
                    if (i < B * R / 4) reinterpret_cast<float4 *>(act)[i] = v[k];
                }
            }
        } else if (LD == 1) {
            for (int c = wave * 256; c < B * R; c += kThreads * 4)
                __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)(cur + c + lane * 4),
                                                 (__attribute__((address_space(3))) void *)(act + c), 16, 0, 16);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {   // fresh address every round: plain (L2-cached) DMA
            for (int c = wave * 256; c < B * R; c += kThreads * 4)
                __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)(cur + c + lane * 4),
                                                 (__attribute__((address_space(3))) void *)(act + c), 16, 0, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        // verify every word: element (b, j) of producer j / U holds r + b + j % U
        unsigned bad = 0;
        if (V) for (int i = tid; i < B * R; i += kThreads) {
            const int b = i / R, j = i - b * R;
            bad += act[i] != (float)(r + b + (j % U));
        }
        if (bad) atomicAdd(reinterpret_cast<unsigned *>(sink), bad);
        acc += act[(tid * 7) % (B * R)];
        __syncthreads();
    }
    if (tid == 0) out[w] = __builtin_amdgcn_s_memrealtime() - t0;
    sink[1 + w] = acc;
}

template <int SIG, int LD, int V>
void run(int G, int B) {
    float *buf, *sink;
    unsigned *ctr, *flags;
    unsigned long long *out;
    const size_t nbuf = (LD == 2 ? 2000ull : 2ull) * B * R;
    hipMalloc(&buf, nbuf * 4);
    hipMalloc(&ctr, kReps * kRepStride * 4);
    hipMalloc(&flags, G * 64);
    hipMalloc(&out, G * 8);
    hipMalloc(&sink, (G + 1) * 4);
    hipMemset(ctr, 0, kReps * kRepStride * 4);
    hipMemset(flags, 0, G * 64);
    hipMemset(sink, 0, (G + 1) * 4);
    hipMemset(buf, 0xFF, nbuf * 4);
    const int rounds = 2000;
    hipFuncSetAttribute((const void *)bulk<SIG, LD, V>, hipFuncAttributeMaxDynamicSharedMemorySize, B * R * 4);
    hipLaunchKernelGGL((bulk<SIG, LD, V>), dim3(G), dim3(kThreads), B * R * 4, 0, buf, ctr, flags, B, rounds, out, sink);
    hipError_t e = hipDeviceSynchronize();
    unsigned long long h[256];
    hipMemcpy(h, out, G * 8, hipMemcpyDeviceToHost);
    unsigned bad = 0;
    hipMemcpy(&bad, sink, 4, hipMemcpyDeviceToHost);
    unsigned long long mx = 0;
    for (int i = 0; i < G; ++i) mx = h[i] > mx ? h[i] : mx;
    printf("%s %s%s G=%3d B=%3d: %.3f us/round  stale=%u  %s\n", SIG == 0 ? "counter" : "flags  ", LD == 0 ? "regs" : LD == 1 ? "dma " : "fresh", V ? " verify" : "", G, B,
           mx * 10e-3 / rounds, bad, hipGetErrorString(e));
    fflush(stdout);
    hipFree(buf); hipFree(ctr); hipFree(flags); hipFree(out); hipFree(sink);
}

int main() {
    for (int B : {1, 4, 16, 32, 64}) {
        run<1, 1, 0>(256, B);
        run<1, 2, 0>(256, B);
        run<1, 2, 1>(256, B);
    }
    return 0;
}
