// cf2sim_rng.h -- Philox4x32-10 counter RNG and Box-Muller normals shared by the HIP kernels
// (the same stream as oracle/cf2_oracle.c).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cf2 {

struct U4 { uint32_t x, y, z, w; };

// Round keys k + r * (W0, W1).  Wave-uniform, so they live in SGPRs (an SGPR operand of v_xor
// costs nothing).  Two forms, chosen per kernel:
//   Keys      all 20 round keys built once per kernel (the env-step kernels).  When the kernel's
//             SGPR budget is exhausted some are spilled to VGPR lanes (a v_readlane per use);
//             -DCF2_VGPR_KEYS holds them in VGPRs instead.
//   KeysBase  only the two base words; each philox() call re-derives its round keys from an
//             opaque copy (2 SALU per round).  Removes the key spills (SGPR spill sites 72 -> 32
//             in the step kernel), but the SALU adds sit in the dependent Philox chain: measured
//             +0.9 us at 262 144 envs and +2k cycles on a lone env wave's physics at 4096 envs;
//             in the register-bound fused rollout it removes the VGPR spills and is still slower
//             (rollout_kernel, CF2_ROLL_BASE_KEYS).  Kept for A/B builds.
struct Keys { uint32_t k0[10], k1[10]; };
__device__ __forceinline__ Keys make_keys(uint32_t k0, uint32_t k1) {
    Keys K;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t a = k0 + (uint32_t)r * 0x9E3779B9u, b = k1 + (uint32_t)r * 0xBB67AE85u;
#ifdef CF2_VGPR_KEYS
        asm volatile("v_mov_b32 %0, %1" : "=v"(K.k0[r]) : "s"(a));
        asm volatile("v_mov_b32 %0, %1" : "=v"(K.k1[r]) : "s"(b));
#else
        K.k0[r] = a; K.k1[r] = b;
#endif
    }
    return K;
}
struct KeysBase { uint32_t k0, k1; };
__device__ __forceinline__ KeysBase make_keys_base(uint32_t k0, uint32_t k1) { return KeysBase{k0, k1}; }
__device__ __forceinline__ Keys make_keys_as(const Keys*, uint32_t k0, uint32_t k1) { return make_keys(k0, k1); }
__device__ __forceinline__ KeysBase make_keys_as(const KeysBase*, uint32_t k0, uint32_t k1) {
    return make_keys_base(k0, k1);
}

#ifndef CF2_PHILOX_ROUNDS
#define CF2_PHILOX_ROUNDS 10   // diagnostic knob only: the stream (and parity) is defined for 10
#endif
__device__ __forceinline__ void philox_round(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t ka,
                                             uint32_t kb) {
    // one v_mad_u64_u32 per product yields both halves
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    // three-input XOR in one v_bitop3_b32 (gfx950; truth table 0x96)
    const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, ka, 0x96);
    const uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, kb, 0x96);
    c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
}
__device__ __forceinline__ U4 philox(const Keys& K, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
#pragma unroll
    for (int r = 0; r < CF2_PHILOX_ROUNDS; ++r) philox_round(c0, c1, c2, c3, K.k0[r], K.k1[r]);
    return U4{c0, c1, c2, c3};
}
__device__ __forceinline__ U4 philox(const KeysBase& K, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
    // opaque per call: the round keys are not common subexpressions of different philox() calls
    uint32_t b0 = K.k0, b1 = K.k1;
    asm volatile("" : "+s"(b0), "+s"(b1));
#pragma unroll
    for (int r = 0; r < CF2_PHILOX_ROUNDS; ++r)
        philox_round(c0, c1, c2, c3, b0 + (uint32_t)r * 0x9E3779B9u, b1 + (uint32_t)r * 0xBB67AE85u);
    return U4{c0, c1, c2, c3};
}

__device__ __forceinline__ float u01(uint32_t x) { return (float)(x >> 8) * 5.9604644775390625e-08f; }

// Box-Muller on the hardware transcendental unit: v_log_f32 is log2, v_sin/v_cos_f32 take
// their argument in revolutions, so sin(2 pi u2) needs no range reduction at all.
__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, float& z0, float& z1) {
    const float u1 = ((float)(a >> 8) + 1.0f) * 5.9604644775390625e-08f;
    const float u2 = (float)(b >> 8) * 5.9604644775390625e-08f;
    const float r = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));  // -2 ln2 log2(u1)
    z0 = r * __builtin_amdgcn_cosf(u2);
    z1 = r * __builtin_amdgcn_sinf(u2);
}

}  // namespace cf2
