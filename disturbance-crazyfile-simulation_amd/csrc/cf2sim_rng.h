// cf2sim_rng.h -- Philox4x32-10 counter RNG and Box-Muller normals shared by the HIP kernels
// (the same stream as oracle/cf2_oracle.c).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cf2 {

struct U4 { uint32_t x, y, z, w; };

// Round keys k + r * (W0, W1), all 20 built once per kernel.  Wave-uniform, so they live in SGPRs
// (an SGPR operand of v_xor costs nothing); when a kernel's SGPR budget is exhausted some are
// spilled to VGPR lanes (a v_readlane per use).  Re-deriving them per call instead (2 SALU per
// round) removed those spills but was slower everywhere it was measured (+0.9 us at 262 144 envs,
// +2 us per env-step in the fused rollout): the SALU adds sit in the dependent Philox chain.
struct Keys { uint32_t k0[10], k1[10]; };
__device__ __forceinline__ Keys make_keys(uint32_t k0, uint32_t k1) {
    Keys K;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        K.k0[r] = k0 + (uint32_t)r * 0x9E3779B9u;
        K.k1[r] = k1 + (uint32_t)r * 0xBB67AE85u;
    }
    return K;
}

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
    for (int r = 0; r < 10; ++r) philox_round(c0, c1, c2, c3, K.k0[r], K.k1[r]);
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
