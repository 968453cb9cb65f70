// mfma_device.h — fp32 MFMA helpers of the register-resident weight kernels (fatchord_xcdm.hip,
// deepmind_xcd.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "wrnn_device.h"

namespace wrnn {

// v_mfma_f32_4x4x1_16b_f32 as inline asm, so that the weights (A) stay where they are: most of
// them in AGPRs, read by the MFMA directly ("a"), the rest in VGPRs — with the builtin, hipcc
// keeps the weights in AGPRs and copies each one to a VGPR (v_accvgpr_read) in front of its MFMA.  Hazards the compiler cannot see inside asm: the
// accumulator chain is dst == srcC (back-to-back, no wait states); the first MFMA of a chain
// takes srcC = 0 (no VALU-written input); the weights are written once, before the loop; the B
// operands come straight from ds_read (waitcnt, no wait states); the VALU reads of a finished
// accumulator wait behind mfma_drain's s_nop (which ties the accumulators).
template <bool kAgpr>
__device__ __forceinline__ void mfma_first(f4v &d, float a, float b) {
    if (kAgpr) asm volatile("v_mfma_f32_4x4x1_16b_f32 %0, %1, %2, 0" : "=&v"(d) : "a"(a), "v"(b));
    else asm volatile("v_mfma_f32_4x4x1_16b_f32 %0, %1, %2, 0" : "=&v"(d) : "v"(a), "v"(b));
}
template <bool kAgpr>
__device__ __forceinline__ void mfma_acc(f4v &d, float a, float b) {
    if (kAgpr) asm volatile("v_mfma_f32_4x4x1_16b_f32 %0, %1, %2, %0" : "+v"(d) : "a"(a), "v"(b));
    else asm volatile("v_mfma_f32_4x4x1_16b_f32 %0, %1, %2, %0" : "+v"(d) : "v"(a), "v"(b));
}
// the same for v_mfma_f32_16x16x4_f32 (16 weight rows × 16 batch rows × 4 columns)
template <bool kAgpr>
__device__ __forceinline__ void mfma16_first(f4v &d, float a, float b) {
    if (kAgpr) asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, 0" : "=&v"(d) : "a"(a), "v"(b));
    else asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, 0" : "=&v"(d) : "v"(a), "v"(b));
}
template <bool kAgpr>
__device__ __forceinline__ void mfma16_acc(f4v &d, float a, float b) {
    if (kAgpr) asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(d) : "a"(a), "v"(b));
    else asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(d) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma16_drain_begin() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory"); }

// ≥ 8 wait states between the last MFMA writing an accumulator and any VALU read of it: one
// s_nop pair, then an empty asm per accumulator that "redefines" it (volatile asm keep their
// order, so every read of the accumulator comes after the nops)
__device__ __forceinline__ void mfma_drain_begin() { asm volatile("s_nop 7\n\ts_nop 1" ::: "memory"); }
__device__ __forceinline__ void mfma_tie(f4v &a) { asm volatile("" : "+v"(a)); }

}  // namespace wrnn
