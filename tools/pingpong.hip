// pingpong.hip — one-way hand-off latency between two workgroups for several store / load
// flavours (the building block of every WaveRNN hop).  WG0 and WG1 alternately write a
// round counter into their own 8-byte word and wait for the other's.  µs per round trip / 2.
//   hipcc --offload-arch=gfx950 -O3 tools/pingpong.hip -o pingpong && ./pingpong
#include <hip/hip_runtime.h>

#include <cstdio>

enum St { ST_RLX_AGENT, ST_RLX_SYSTEM, ST_XCHG_AGENT, ST_STORE_WBL2, ST_ATOMIC_ADD };
enum Ld { LD_RLX_AGENT, LD_RLX_SYSTEM, LD_FETCH_ADD0, LD_ACQ_FENCE };
static const char *stn[] = {"store rlx agent (sc1)", "store rlx system", "xchg agent", "store+wbl2", "atomic add"};
static const char *ldn[] = {"load rlx agent (sc1)", "load rlx system", "fetch_add 0", "plain+acq fence"};

template <int ST, int LD>
__global__ void pp(unsigned long long *w, int rounds, unsigned long long *out, int stride) {
    if (threadIdx.x != 0) return;
    const int me = blockIdx.x, other = 1 - me;
    unsigned long long *mine = w + me * stride, *theirs = w + other * stride;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int r = 1; r <= rounds; ++r) {
        if (me == 1 || r > 1) {
            // wait for the other's value r (WG1) or r-1 (WG0)
            const unsigned long long want = me == 1 ? r : r - 1;
            for (;;) {
                unsigned long long v;
                if (LD == LD_RLX_AGENT) v = __hip_atomic_load(theirs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else if (LD == LD_RLX_SYSTEM) v = __hip_atomic_load(theirs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                else if (LD == LD_FETCH_ADD0) v = __hip_atomic_fetch_add(theirs, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent"); v = *(volatile unsigned long long *)theirs; }
                if (v >= want) break;
            }
        }
        if (ST == ST_RLX_AGENT) __hip_atomic_store(mine, (unsigned long long)r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else if (ST == ST_RLX_SYSTEM) __hip_atomic_store(mine, (unsigned long long)r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        else if (ST == ST_XCHG_AGENT) (void)__hip_atomic_exchange(mine, (unsigned long long)r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else if (ST == ST_STORE_WBL2) {
            *(volatile unsigned long long *)mine = r;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        } else (void)__hip_atomic_fetch_add(mine, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    out[me] = __builtin_amdgcn_s_memrealtime() - t0;
}

// Symmetric exchange: both workgroups publish round r, then wait for the other's round r.
// MODE 0: one wave, lane 0 does both; MODE 1: + a 4-wave s_barrier per round;
// MODE 2: wave 3 publishes, wave 0 polls, 4-wave s_barrier per round.
template <int MODE>
__global__ __launch_bounds__(256) void xchg(unsigned long long *w, int rounds, unsigned long long *out, int stride) {
    const int me = blockIdx.x, other = 1 - me, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    unsigned long long *mine = w + me * stride, *theirs = w + other * stride;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int r = 1; r <= rounds; ++r) {
        const int pub_wave = MODE == 2 ? 3 : 0;
        if (wave == pub_wave && lane == 0)
            __hip_atomic_store(mine, (unsigned long long)r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (wave == 0 && lane == 0)
            while (__hip_atomic_load(theirs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned long long)r) {}
        if (MODE >= 1) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        }
    }
    if (threadIdx.x == 0) out[me] = __builtin_amdgcn_s_memrealtime() - t0;
}

// Bisect xchg (0.7 us) → hopbench (1.45 us):
// V 0: poll only the other's word; 1: poll own + other's word (same line, adjacent)
// 2: as 1 but the words 512 B apart; 3: as 1 with two lanes polling one word each
template <int V>
__global__ __launch_bounds__(256) void xchg2(unsigned long long *w, int rounds, unsigned long long *out) {
    const int me = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int sp = V == 2 ? 64 : 1;
    unsigned long long *mine = w + me * sp;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int r = 1; r <= rounds; ++r) {
        if (wave == 3 && lane == 0) __hip_atomic_store(mine, (unsigned long long)r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (wave == 0) {
            if (V == 0) {
                if (lane == 0) while (__hip_atomic_load(w + (1 - me) * sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned long long)r) {}
            } else if (V == 3) {
                if (lane < 2) while (__hip_atomic_load(w + lane * sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned long long)r) {}
            } else if (lane == 0) {
                for (;;) {
                    unsigned long long a = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    unsigned long long b = __hip_atomic_load(w + sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (a >= (unsigned long long)r && b >= (unsigned long long)r) break;
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    }
    if (threadIdx.x == 0) out[me] = __builtin_amdgcn_s_memrealtime() - t0;
}

template <int V>
void runx2(unsigned long long *w, unsigned long long *out) {
    const int rounds = 2000;
    hipMemset(w, 0, 1 << 20);
    hipLaunchKernelGGL((xchg2<V>), dim3(2), dim3(256), 0, 0, w, rounds, out);
    hipDeviceSynchronize();
    unsigned long long h[2];
    hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
    printf("bisect V%d: %.3f us per round\n", V, (h[0] > h[1] ? h[0] : h[1]) * 10e-3 / rounds);
    fflush(stdout);
}

template <int MODE>
void runx(unsigned long long *w, unsigned long long *out, int threads) {
    const int rounds = 2000;
    hipMemset(w, 0, 1 << 20);
    hipLaunchKernelGGL((xchg<MODE>), dim3(2), dim3(threads), 0, 0, w, rounds, out, 64);
    hipDeviceSynchronize();
    unsigned long long h[2];
    hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
    printf("exchange mode %d (%d threads): %.3f us per round\n", MODE, threads, (h[0] > h[1] ? h[0] : h[1]) * 10e-3 / rounds);
    fflush(stdout);
}

template <int ST, int LD>
void run(unsigned long long *w, unsigned long long *out, int stride) {
    const int rounds = 2000;
    hipMemset(w, 0, 1 << 20);
    hipLaunchKernelGGL((pp<ST, LD>), dim3(2), dim3(64), 0, 0, w, rounds, out, stride);
    hipDeviceSynchronize();
    unsigned long long h[2];
    hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
    const double us = (h[0] > h[1] ? h[0] : h[1]) * 10e-3 / rounds / 2;
    printf("%-24s %-22s stride %5d B: %.3f us one-way\n", stn[ST], ldn[LD], stride * 8, us);
    fflush(stdout);
}

int main() {
    unsigned long long *w, *out;
    hipMalloc(&w, 1 << 20);
    hipMalloc(&out, 64);
    runx2<0>(w, out);
    runx2<1>(w, out);
    runx2<2>(w, out);
    runx2<3>(w, out);
    runx<0>(w, out, 64);
    runx<0>(w, out, 256);
    runx<1>(w, out, 256);
    runx<2>(w, out, 256);
    for (int stride : {8}) {
        run<ST_RLX_AGENT, LD_RLX_AGENT>(w, out, stride);
        run<ST_RLX_SYSTEM, LD_RLX_AGENT>(w, out, stride);
        run<ST_RLX_AGENT, LD_RLX_SYSTEM>(w, out, stride);
        run<ST_XCHG_AGENT, LD_RLX_AGENT>(w, out, stride);
        run<ST_ATOMIC_ADD, LD_RLX_AGENT>(w, out, stride);
        run<ST_RLX_AGENT, LD_FETCH_ADD0>(w, out, stride);
        run<ST_XCHG_AGENT, LD_FETCH_ADD0>(w, out, stride);
        run<ST_STORE_WBL2, LD_ACQ_FENCE>(w, out, stride);
        run<ST_STORE_WBL2, LD_RLX_AGENT>(w, out, stride);
    }
    return 0;
}
