// cf2sim_kernels.hip -- fused CDNA4 (gfx950) env-step / reset kernels for the batched
// CrazyFlie hover environment.
//
// One lane = one env.  Env state is AoSoA in HBM: tiles of 64 envs (one wave), each env's 480 B
// as 30 float4 groups, group g of lane l at tile_base + g * 1024 + l * 16 (cf2sim_internal.h,
// DESIGN.md section 2), so every state access of a wave is one coalesced 1-KB dwordx4 transaction.
// A step loads the state once, runs aggregate_phy_steps physics sub-steps plus the
// observation / history / reward / done epilogue (and the auto-reset of finished envs) in
// registers, and stores the state once: the kernel is HBM-bound by construction (no MFMA:
// the work is per-env element-wise, not a contraction).
//
// What each piece restates (reference paths, phoenix_drone_simulation/ omitted):
//   apply_action            envs/agents.py:259-298, envs/control.py:94-100, envs/utils.py:130-134
//   force/torque assembly   envs/physics.py:213-250, envs/agents.py:300-337,517-533
//   rigid-body step         bullet3 3.21 btMultiBody (third party; see oracle/cf2_oracle.c header)
//   SimplePhysics           envs/physics.py:130-200
//   update_information      envs/agents.py:434-453
//   compute_observation     envs/hover_free.py:168-200, envs/sensors.py:75-134, envs/utils.py:102-105
//   compute_history         envs/base.py:305-321
//   reward / done / cost    envs/hover_free.py:124-235,449-461, envs/hover.py:102-202
//   reset + DR              envs/base.py:241-298,420-464, envs/hover_free.py:237-289
//   HJ disturbance          adversarial_generation/FasTrack_data/distur_gener.py:19-207,
//                           adversarial_generation/odp/Grid/GridProcessing.py:52-71
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "cf2sim_internal.h"
#include "cf2sim_rng.h"
#include "cf2sim_policy.h"

namespace cf2 {

// Random-word sources: Rng computes Philox blocks; TableRng reads blocks a whole block of
// threads precomputed into LDS (auto-reset, see step_kernel).  Counter = (block, rng counter,
// global env id, tag).
template <class KT>
struct RngT {
    const KT& K;
    uint32_t ctr, gid, tag;
    __device__ __forceinline__ U4 block(uint32_t b) const { return philox(K, b, ctr, gid, tag); }
};
using Rng = RngT<Keys>;

// reset-time blocks (reset_env): 0-13 direct, sensor calls at 32-37 and 40-45
enum { RESET_SLOTS = 26 };
__host__ __device__ constexpr int reset_slot(uint32_t b) { return b < 14 ? (int)b : (b < 40 ? 14 + (int)b - 32 : 20 + (int)b - 40); }
__host__ __device__ constexpr uint32_t reset_block_of_slot(int s) { return s < 14 ? (uint32_t)s : (s < 20 ? 32u + (uint32_t)(s - 14) : 40u + (uint32_t)(s - 20)); }

struct TableRng {
    const uint32_t* t;      // LDS: word w of slot s at t[(s * 4 + w) * stride]
    uint32_t stride;
    __device__ __forceinline__ U4 block(uint32_t b) const {
        const uint32_t* q = t + (size_t)reset_slot(b) * 4 * stride;
        return U4{q[0], q[stride], q[2 * stride], q[3 * stride]};
    }
};

// N normals from consecutive blocks starting at b0 (pair k uses u32 2k, 2k+1)
template <int N, class G>
__device__ __forceinline__ void normals(const G& g, uint32_t b0, float (&z)[N]) {
#pragma unroll
    for (int blk = 0; blk < (N + 3) / 4; ++blk) {
        const U4 u = g.block(b0 + blk);
        float a0, a1, a2, a3;
        box_muller(u.x, u.y, a0, a1);
        if (4 * blk + 0 < N) z[4 * blk + 0] = a0;
        if (4 * blk + 1 < N) z[4 * blk + 1] = a1;
        if (4 * blk + 2 < N) {
            box_muller(u.z, u.w, a2, a3);
            z[4 * blk + 2] = a2;
            if (4 * blk + 3 < N) z[4 * blk + 3] = a3;
        }
    }
}

// The auto-reset table holds the Box-Muller outputs, not the raw words, of the word pairs the
// reset turns into normals (reset_env: blocks 4-8; its two sensor calls: blocks 32-35 and 40-43
// whole, 36 and 44 first pair).  They are transformed block-parallel while the table is drawn,
// which takes ~110 transcendentals off the one-lane-per-env reset path.
__host__ __device__ constexpr bool reset_slot_normal_xy(int s) {
    return (s >= 4 && s <= 8) || (s >= 14 && s <= 18) || (s >= 20 && s <= 24);
}
__host__ __device__ constexpr bool reset_slot_normal_zw(int s) {
    return (s >= 4 && s <= 8) || (s >= 14 && s <= 17) || (s >= 20 && s <= 23);
}
template <int N>
__device__ __forceinline__ void normals(const TableRng& g, uint32_t b0, float (&z)[N]) {
#pragma unroll
    for (int blk = 0; blk < (N + 3) / 4; ++blk) {
        const U4 u = g.block(b0 + blk);
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (4 * blk + k < N) z[4 * blk + k] = __uint_as_float(w[k]);
    }
}

// The final sensor call's six Philox blocks, drawn while the env's state is still in flight and
// parked in the lane's own LDS obs-staging row (which the observation overwrites only after the
// call): row words 0-17 are the call's 18 normals (Box-Muller already applied), 18-23 the raw words
// of its uniforms.  block(b) returns row words 4(b-b0)..+3, normals<N> the first N row words.
// STRIDE: distance between consecutive words (1: the lane's own LDS row; 64: a [word][env] table
// of the small-N kernel, where the helper waves stage the env-step's later draws)
template <uint32_t STRIDE = 1>
struct RowRng {
    const uint32_t* t;
    uint32_t b0;
    __device__ __forceinline__ U4 block(uint32_t b) const {
        const uint32_t* q = t + 4u * (b - b0) * STRIDE;
        return U4{q[0], q[STRIDE], q[2 * STRIDE], q[3 * STRIDE]};
    }
};
template <int N, uint32_t STRIDE>
__device__ __forceinline__ void normals(const RowRng<STRIDE>& g, uint32_t b0, float (&z)[N]) {
#pragma unroll
    for (int k = 0; k < N; ++k) z[k] = __uint_as_float(g.t[(4u * (b0 - g.b0) + k) * STRIDE]);
}

// The small-N kernel's helper-drawn env-step randomness ([word][env] in LDS, stride 64): what the
// env-step draws from its first sensor call on in the reference-default shape (SPEC 1 with sensor
// noise), with Box-Muller already applied to the words that become normals:
//   words  0-3   OU normals of sub-step 1              (step block 2)
//   words  4-12  gyro normals of sub-step 1's call      (normals<9> at block 16: blocks 16-18)
//   words 13-30  final sensor call's 18 normals         (normals<18> at block 24: blocks 24-28)
//   words 31-36  its uniform words: block 28 .z .w, block 29 .x .y .z .w
//   words 37-45  gyro normals 6-14 of sub-step 0's call (normals_range<6, 15> at block 8: blocks 9-11;
//                the call is a full one whose held part is dead, compute_observation)
// The env wave joins the helpers' LDS barrier before that first sensor call.
enum { HD_WORDS = 46, HD_OU1 = 0, HD_GYRO1 = 4, HD_FINAL = 13, HD_GYRO0 = 37 };

// Normals LO..HI-1 of the sequence normals<N>(g, b0, .) would produce, drawing only the Philox
// blocks and Box-Muller pairs that cover them (the stream positions of all other draws are
// unchanged, so skipping dead draws is invisible to everything else).
template <int LO, int HI, class G>
__device__ __forceinline__ void normals_range(const G& g, uint32_t b0, float* z) {
#pragma unroll
    for (int blk = LO / 4; blk < (HI + 3) / 4; ++blk) {
        const U4 u = g.block(b0 + blk);
        float a[4];
        if (4 * blk + 1 >= LO && 4 * blk < HI) box_muller(u.x, u.y, a[0], a[1]);
        if (4 * blk + 3 >= LO && 4 * blk + 2 < HI) box_muller(u.z, u.w, a[2], a[3]);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (4 * blk + k >= LO && 4 * blk + k < HI) z[4 * blk + k] = a[k];
    }
}

// (the reset table already holds the Box-Muller outputs of its normal slots)
template <int LO, int HI>
__device__ __forceinline__ void normals_range(const TableRng& g, uint32_t b0, float* z) {
#pragma unroll
    for (int blk = LO / 4; blk < (HI + 3) / 4; ++blk) {
        const U4 u = g.block(b0 + blk);
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (4 * blk + k >= LO && 4 * blk + k < HI) z[4 * blk + k] = __uint_as_float(w[k]);
    }
}

// The small-N kernels' helper waves 1-3 draw the env-step's randomness of the HD_* layout for the
// env of their lane (d = its column of the [word][env] LDS table, stride 64), the step counter ctr
// known from the state.  Sub-step 0's gyro normals first: the env wave needs them earliest.
__device__ __forceinline__ void helper_step_draws(const Keys& K, uint32_t ctr, uint32_t gid, uint32_t wave, float* d) {
    const RngT<Keys> g{K, ctr, gid, TAG_STEP};
    auto bm4 = [&](uint32_t blk, int w) {          // 4 normals of one block -> words w..w+3
        const U4 u = g.block(blk);
        float z0, z1, z2, z3;
        box_muller(u.x, u.y, z0, z1);
        box_muller(u.z, u.w, z2, z3);
        d[(w + 0) * 64] = z0; d[(w + 1) * 64] = z1; d[(w + 2) * 64] = z2; d[(w + 3) * 64] = z3;
    };
    if (wave == 1) {
        bm4(2, HD_OU1);                             // OU of sub-step 1
        bm4(16, HD_GYRO1);                          // sub-step 1 sensor call: normals 0-8
        bm4(17, HD_GYRO1 + 4);
        const U4 u = g.block(18);
        float z0, z1;
        box_muller(u.x, u.y, z0, z1);
        d[(HD_GYRO1 + 8) * 64] = z0;
    } else if (wave == 2) {
        {
            const U4 u = g.block(9);                // sub-step 0 sensor call: normals 6-7
            float z2, z3;
            box_muller(u.z, u.w, z2, z3);
            d[(HD_GYRO0 + 0) * 64] = z2; d[(HD_GYRO0 + 1) * 64] = z3;
        }
        bm4(24, HD_FINAL);                          // final sensor call: normals 0-11
        bm4(25, HD_FINAL + 4);
        bm4(26, HD_FINAL + 8);
    } else {
        bm4(10, HD_GYRO0 + 2);                      // sub-step 0 sensor call: normals 8-11
        {
            const U4 u = g.block(11);               // normals 12-14
            float z0, z1, z2, z3;
            box_muller(u.x, u.y, z0, z1);
            box_muller(u.z, u.w, z2, z3);
            d[(HD_GYRO0 + 6) * 64] = z0; d[(HD_GYRO0 + 7) * 64] = z1; d[(HD_GYRO0 + 8) * 64] = z2;
            (void)z3;
        }
        bm4(27, HD_FINAL + 12);                     // normals 12-15
        const U4 u = g.block(28), v = g.block(29);
        float z0, z1;
        box_muller(u.x, u.y, z0, z1);               // normals 16-17, then the six uniform words
        d[(HD_FINAL + 16) * 64] = z0; d[(HD_FINAL + 17) * 64] = z1;
        d[(HD_FINAL + 18) * 64] = __uint_as_float(u.z); d[(HD_FINAL + 19) * 64] = __uint_as_float(u.w);
        d[(HD_FINAL + 20) * 64] = __uint_as_float(v.x); d[(HD_FINAL + 21) * 64] = __uint_as_float(v.y);
        d[(HD_FINAL + 22) * 64] = __uint_as_float(v.z); d[(HD_FINAL + 23) * 64] = __uint_as_float(v.w);
    }
}

// ------------------------------------------------------------------------------------
// rotation helpers (PyBullet C-API semantics)
// ------------------------------------------------------------------------------------
// DIV_NOTE: a division by a constant, x / c, is compiled (fp32, -fno-hip-fp32-correctly-rounded-
// divide-sqrt) as frexp(x), mantissa * rn(1 / c) scaled to [1, 2), ldexp: five VALU, and for every
// normal x bit-identical to x * rn(1 / c) (scaling by a power of two commutes with rounding), which
// is one.  The env-step divides by constants 19 times (PWM, rpm, the done test): written as products.
// v_rcp_f32 / v_rsq_f32 (1 ulp) for well-scaled operands (no denormal pre-scaling)
__device__ __forceinline__ float rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float rsq(float x) { return __builtin_amdgcn_rsqf(x); }

struct M3 { float m[9]; };

__device__ __forceinline__ M3 rotmat(const float q[4]) {
    const float x = q[0], y = q[1], z = q[2], w = q[3];
    const float d = x * x + y * y + z * z + w * w;
    const float s = 2.0f * rcp(d);
    const float xs = x * s, ys = y * s, zs = z * s;
    const float wx = w * xs, wy = w * ys, wz = w * zs;
    const float xx = x * xs, xy = x * ys, xz = x * zs;
    const float yy = y * ys, yz = y * zs, zz = z * zs;
    M3 r;
    r.m[0] = 1.0f - (yy + zz); r.m[1] = xy - wz;          r.m[2] = xz + wy;
    r.m[3] = xy + wz;          r.m[4] = 1.0f - (xx + zz); r.m[5] = yz - wx;
    r.m[6] = xz - wy;          r.m[7] = yz + wx;          r.m[8] = 1.0f - (xx + yy);
    return r;
}
__device__ __forceinline__ void mv(const M3& R, const float v[3], float o[3]) {
    o[0] = R.m[0] * v[0] + R.m[1] * v[1] + R.m[2] * v[2];
    o[1] = R.m[3] * v[0] + R.m[4] * v[1] + R.m[5] * v[2];
    o[2] = R.m[6] * v[0] + R.m[7] * v[1] + R.m[8] * v[2];
}
__device__ __forceinline__ void mtv(const M3& R, const float v[3], float o[3]) {
    o[0] = R.m[0] * v[0] + R.m[3] * v[1] + R.m[6] * v[2];
    o[1] = R.m[1] * v[0] + R.m[4] * v[1] + R.m[7] * v[2];
    o[2] = R.m[2] * v[0] + R.m[5] * v[1] + R.m[8] * v[2];
}
// v_sqrt_f32 without the denormal pre-scaling sqrtf adds (6 instructions -> 1): the same result
// for every normal operand; a denormal operand (|v| < 1e-19) gives 0
__device__ __forceinline__ float sqrt_fast(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float norm3(const float v[3]) { return sqrt_fast(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }
// clip(x, lo, hi) for lo <= hi as one v_med3_f32 (identical to the compare form for non-NaN x)
__device__ __forceinline__ float clampf(float x, float lo, float hi) { return __builtin_amdgcn_fmed3f(x, lo, hi); }
// Makes a register value opaque to the optimiser.  Used before data-dependent selects among
// Env fields: otherwise InstCombine turns select(c, load p, load q) chains into a load of a
// select of pointers, SROA can no longer promote the Env struct and it lands in scratch.
__device__ __forceinline__ float opaque(float x) { asm("" : "+v"(x)); return x; }

// ---- short-range elementary functions (VALU polynomials instead of the ocml library paths,
// whose general range reduction costs ~100 instructions each).  Errors are a few fp32 ulp.
// sin and cos of x: Cody-Waite reduction by pi/2 (3-part constant, exact for |x| < ~1e4), then
// degree-11/12 Taylor polynomials on [-pi/4, pi/4] (truncation < 2e-9)
__device__ __forceinline__ void sincos_fast(float x, float& s, float& c) {
    const float k = __builtin_rintf(x * 0.63661977236758134f);
    float r = __builtin_fmaf(k, -1.5707963705062866f, x);
    r = __builtin_fmaf(k, 4.3711388286737929e-08f, r);
    r = __builtin_fmaf(k, 1.7151245100059206e-15f, r);
    const float r2 = r * r;
    const float sr = r * (1.0f + r2 * (-1.6666667e-1f + r2 * (8.3333333e-3f + r2 * (-1.9841270e-4f + r2 * (2.7557319e-6f - r2 * 2.5052108e-8f)))));
    const float cr = 1.0f + r2 * (-0.5f + r2 * (4.1666668e-2f + r2 * (-1.3888889e-3f + r2 * (2.4801587e-5f + r2 * (-2.7557319e-7f + r2 * 2.0876757e-9f)))));
    const int q = (int)k & 3;
    const float ss = (q & 1) ? cr : sr, cc = (q & 1) ? sr : cr;
    s = (q & 2) ? -ss : ss;
    c = ((q + 1) & 2) ? -cc : cc;
}
// atan2 (Cephes atanf kernel on the reduced ratio min/max in [0, 1], reduced again about 1)
__device__ __forceinline__ float atan2_fast(float y, float x) {
    const float ax = fabsf(x), ay = fabsf(y);
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    float t = mx > 0.0f ? mn * rcp(mx) : 0.0f;
    const bool red = t > 0.41421356237309503f;
    const float z = red ? (t - 1.0f) * rcp(t + 1.0f) : t;
    const float z2 = z * z;
    float r = (((8.05374449538e-2f * z2 - 1.38776856032e-1f) * z2 + 1.99777106478e-1f) * z2 - 3.33329491539e-1f) * z2 * z + z;
    r = red ? r + 0.78539816339744831f : r;
    r = ay > ax ? 1.5707963267948966f - r : r;
    r = x < 0.0f ? 3.1415926535897932f - r : r;
    return __builtin_copysignf(r, y);
}
__device__ __forceinline__ float asin_fast(float x) {
    return atan2_fast(x, sqrt_fast(fmaxf(0.0f, (1.0f - x) * (1.0f + x))));
}

__device__ __forceinline__ void quat_from_euler(const float e[3], float q[4]) {
    const float phi = e[0] * 0.5f, the = e[1] * 0.5f, psi = e[2] * 0.5f;
    float sp, cp, st, ct, ss, cs;
    sincos_fast(phi, sp, cp);
    sincos_fast(the, st, ct);
    sincos_fast(psi, ss, cs);
    const float x = sp * ct * cs - cp * st * ss;
    const float y = cp * st * cs + sp * ct * ss;
    const float z = cp * ct * ss - sp * st * cs;
    const float w = cp * ct * cs + sp * st * ss;
    const float il = rsq(x * x + y * y + z * z + w * w);
    q[0] = x * il; q[1] = y * il; q[2] = z * il; q[3] = w * il;
}
// the observation's quaternion of the noisy rpy (sensors.py): sin/cos on the transcendental unit
// (v_sin/v_cos take revolutions), 3 muls + 6 quarter-rate ops instead of ~75 polynomial VALU ops
__device__ __forceinline__ void quat_from_euler_obs(const float e[3], float q[4]) {
    constexpr float inv4pi = 0.079577471545947668f;     // half angle in revolutions: e / 2 / (2 pi)
    const float phi = e[0] * inv4pi, the = e[1] * inv4pi, psi = e[2] * inv4pi;
    const float sp = __builtin_amdgcn_sinf(phi), cp = __builtin_amdgcn_cosf(phi);
    const float st = __builtin_amdgcn_sinf(the), ct = __builtin_amdgcn_cosf(the);
    const float ss = __builtin_amdgcn_sinf(psi), cs = __builtin_amdgcn_cosf(psi);
    const float x = sp * ct * cs - cp * st * ss;
    const float y = cp * st * cs + sp * ct * ss;
    const float z = cp * ct * ss - sp * st * cs;
    const float w = cp * ct * cs + sp * st * ss;
    const float il = rsq(x * x + y * y + z * z + w * w);
    q[0] = x * il; q[1] = y * il; q[2] = z * il; q[3] = w * il;
}
__device__ __forceinline__ void euler_from_quat(const float q[4], float e[3]) {
    const float sqx = q[0] * q[0], sqy = q[1] * q[1], sqz = q[2] * q[2], squ = q[3] * q[3];
    const float sarg = -2.0f * (q[0] * q[2] - q[3] * q[1]);
    // branch-free form of the three cases (gimbal lock at sarg <= -0.99999 / >= 0.99999): the
    // atan2 of the yaw takes case-selected arguments, so each function is evaluated once
    const bool lo = sarg <= -0.99999f, hi = sarg >= 0.99999f, mid = !(lo || hi);
    const float e0 = atan2_fast(2.0f * (q[1] * q[2] + q[3] * q[0]), squ - sqx - sqy + sqz);
    const float e1 = asin_fast(fminf(fmaxf(sarg, -1.0f), 1.0f));
    const float y2 = mid ? 2.0f * (q[0] * q[1] + q[3] * q[2]) : (lo ? q[0] : -q[0]);
    const float x2 = mid ? squ + sqx - sqy - sqz : (lo ? -q[1] : q[1]);
    const float e2 = atan2_fast(y2, x2);
    e[0] = mid ? e0 : 0.0f;
    e[1] = mid ? e1 : (lo ? -0.5f * 3.141592653589793f : 0.5f * 3.141592653589793f);
    e[2] = mid ? e2 : 2.0f * e2;
}
__device__ __forceinline__ void quat2euler(const float q[4], float e[3]) {
    const float x = q[0], y = q[1], z = q[2], w = q[3];
    const float t0 = 2.0f * (w * x + y * z);
    const float t1 = 1.0f - 2.0f * (x * x + y * y);
    e[0] = atan2f(t0, t1);
    float t2 = 2.0f * (w * y - z * x);
    t2 = t2 > 1.0f ? 1.0f : t2;
    t2 = t2 < -1.0f ? -1.0f : t2;
    e[1] = asinf(t2);
    const float t3 = 2.0f * (w * z + x * y);
    const float t4 = 1.0f - 2.0f * (y * y + z * z);
    e[2] = atan2f(t3, t4);
}

// ------------------------------------------------------------------------------------
// HJ value-table gather (7 taps: centre and +-1 along the three rate dims)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ int grid_nearest(const double* pts, double s) {
    // searchsorted(side='left') on the sorted nodes = the number of nodes below s: a branch-free
    // binary search over 16 slots (slot 15 is +inf), 4 compares instead of 15
    static_assert(HJ_PTS == 15, "16-slot search");
    int idx = 0;
#pragma unroll
    for (int step = 8; step >= 1; step >>= 1) {
        const int k = idx + step - 1;
        idx += (k < HJ_PTS && pts[k < HJ_PTS ? k : HJ_PTS - 1] < s) ? step : 0;
    }
    if (idx > 0 && (idx == HJ_PTS || fabs(s - pts[idx - 1]) < fabs(s - pts[idx]))) return idx - 1;
    return idx;
}
__device__ __forceinline__ float sgnf(float v) { return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f); }

// returns bit i set <=> dV/dx_{3+i} > 0 (opt disturbance = -dmax_i).  grid: the 6 x 15 grid
// points (KTables::hj_grid) staged in LDS by the calling kernel: the nearest-node searches then
// cost LDS round trips instead of serialised global loads.
// distur_gener's sign rule at grid node c (flat index) with per-dim indices idx: for each rate
// dimension d = 3..5 the one-sided differences L, R of V around the node (GridProcessing.py
// spatial derivative with the boundary extrapolation of distur_gener.py:160-183), bit d-3 = L > -R
__device__ __forceinline__ unsigned hj_node_bits(const float* __restrict__ V, int c, const int idx[6]) {
    const int stride[6] = {759375, 50625, 3375, 225, 15, 1};
    const float Vc = V[c];
    unsigned bits = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const int d = 3 + i;
        const int s = stride[d];
        float L, Rr;
        if (idx[d] == 0) {
            const float Vn = V[c + s];
            const float lb = __fadd_rn(Vc, __fmul_rn(fabsf(__fsub_rn(Vn, Vc)), sgnf(Vc)));
            L = __fsub_rn(Vc, lb); Rr = __fsub_rn(Vn, Vc);
        } else if (idx[d] == HJ_PTS - 1) {
            const float Vp = V[c - s];
            const float rb = __fadd_rn(Vc, __fmul_rn(fabsf(__fsub_rn(Vc, Vp)), sgnf(Vc)));
            L = __fsub_rn(Vc, Vp); Rr = __fsub_rn(rb, Vc);
        } else {
            const float Vp = V[c - s], Vn = V[c + s];
            L = __fsub_rn(Vc, Vp); Rr = __fsub_rn(Vn, Vc);
        }
        bits |= (L > -Rr ? 1u : 0u) << i;
    }
    return bits;
}
// nearest grid node of a state (Grid.get_index, GridProcessing.py:52-71): flat index and per-dim indices
__device__ __forceinline__ int hj_node(const double st[6], const double* grid, int idx[6]) {
    const int stride[6] = {759375, 50625, 3375, 225, 15, 1};
    int c = 0;
#pragma unroll
    for (int d = 0; d < 6; ++d) {
        idx[d] = grid_nearest(grid + d * HJ_PTS, st[d]);
        c += idx[d] * stride[d];
    }
    return c;
}
__device__ __forceinline__ unsigned hj_signs(const float* __restrict__ V, const double st[6], const double* grid) {
    int idx[6];
    const int c = hj_node(st, grid, idx);
    return hj_node_bits(V, c, idx);
}

// every thread of the block takes part (contains a block barrier)
__device__ __forceinline__ void stage_hj_grid(const double (*src)[HJ_PTS], double* s_grid) {
    for (uint32_t k = threadIdx.x; k < 6u * HJ_PTS; k += blockDim.x) s_grid[k] = src[k / HJ_PTS][k % HJ_PTS];
    __syncthreads();
}

// Coalesced write-out of a block's LDS-staged obs rows (contiguous in global memory) as
// non-temporal stores. The caller reads each row once (policy input, rollout storage), and the nt
// stores keep the rows from displacing the env state in the Infinity Cache between env-steps.
// Same-box A/B at 262 144 envs (tools/ab_rollout_nt.sh): the env-step 39.5 -> 38.5 us with the
// state streaming from HBM and 36.3 -> 36.0 us with it cache-resident; the rollout caller, whose
// policy reads these rows next, unchanged (bf16x3) to 1 % faster (fp32). Non-temporal loads of
// the actions helped the streaming case and cost +2 us in the resident one, so they were not kept.
// The full-block path is unrolled: every LDS read of the thread's chunks is issued before the first
// global store, so the chunks pay one LDS round trip instead of one each (the rolled loop waited
// lgkmcnt(0) before every store: ~3.2k cycles of the small-N env wave for its 9 chunks, r05 timeline).
template <uint32_t EPB, uint32_t OD, uint32_t NT>
__device__ __forceinline__ void write_obs_rows(float* dst, const float* s_obs, uint32_t nvalid, uint32_t tid) {
    typedef float f4x __attribute__((ext_vector_type(4)));
    typedef float f2x __attribute__((ext_vector_type(2)));
    constexpr uint32_t epb = EPB, od = OD, nthreads = NT;
    if ((EPB * OD) % 4 == 0 && nvalid == epb && ((uintptr_t)dst & 15u) == 0) {
        constexpr uint32_t NQ = EPB * OD / 4, IT = (NQ + NT - 1) / NT;
        const f4x* src4 = reinterpret_cast<const f4x*>(s_obs);
        f4x* dst4 = reinterpret_cast<f4x*>(dst);
        f4x v[IT];
#pragma unroll
        for (uint32_t it = 0; it < IT; ++it) {
            const uint32_t k = tid + it * NT;
            v[it] = src4[k < NQ ? k : NQ - 1u];
        }
#pragma unroll
        for (uint32_t it = 0; it < IT; ++it) {
            const uint32_t k = tid + it * NT;
            if (NQ % NT == 0 || k < NQ) __builtin_nontemporal_store(v[it], dst4 + k);
        }
    } else {
        const f2x* src2 = reinterpret_cast<const f2x*>(s_obs);
        f2x* dst2 = reinterpret_cast<f2x*>(dst);
        for (uint32_t k = tid; k < nvalid * od / 2; k += nthreads) __builtin_nontemporal_store(src2[k], dst2 + k);
    }
}

// Block barrier for LDS hand-offs: the calling wave's LDS operations complete first, then
// s_barrier.  (On gfx950 __syncthreads lowers to the same two instructions -- its workgroup-scope
// fence needs no vmcnt wait -- but this form is explicit about what the hand-off relies on, and it
// has no fence semantics the compiler could move memory operations around.)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// A one-way hand-over between waves of a block without a block barrier: the producer's lane 0
// sets an LDS flag after the wave's LDS writes; consumers poll it (bounded, so a flag never set
// cannot hang the grid: the wait then records CF2_DEVERR_HANDOVER in the context's device error
// word, which cf2_device_errors reports, and BatchedCrazyflieEnv.check_device_errors raises on).
__device__ __forceinline__ void lds_flag_set(uint32_t* f) {
    __hip_atomic_store(f, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_flag_wait(uint32_t* f, const KTables* tab) {
    for (uint32_t it = 0; it < (1u << 22); ++it) {
        if (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != 0u) return;
        __builtin_amdgcn_s_sleep(1);
    }
    atomicOr(const_cast<uint32_t*>(&tab->dev_err), (uint32_t)CF2_DEVERR_HANDOVER);
}

// One wave's part of the small-N kernel's write-out of its 64 obs rows: the float4 chunks that touch
// a row whose bit in mask is set (dirty: the reset observations the helper waves staged in rrow) or
// those that do not (from obs, the env-step's observations).  A chunk straddling a reset and a
// non-reset row is a dirty chunk, merged from both.
template <uint32_t OD>
__device__ __forceinline__ void write_obs_rows_part(float* dst, const float* s_obs, const float* s_rrow, uint64_t mask,
                                                    uint32_t nvalid, uint32_t lane, bool dirty) {
    typedef float f4x __attribute__((ext_vector_type(4)));
    typedef float f2x __attribute__((ext_vector_type(2)));
    if (nvalid == 64u && (64u * OD) % 4 == 0 && ((uintptr_t)dst & 15u) == 0) {
        // unrolled: the chunks' LDS reads all issue before the first store (one LDS round trip)
        constexpr uint32_t NQ = 64u * OD / 4, IT = (NQ + 63u) / 64u;
        const f4x* a4 = reinterpret_cast<const f4x*>(s_obs);
        const f4x* b4 = reinterpret_cast<const f4x*>(s_rrow);
        f4x* dst4 = reinterpret_cast<f4x*>(dst);
        f4x v[IT];
        bool on[IT];
#pragma unroll
        for (uint32_t it = 0; it < IT; ++it) {
            const uint32_t k = lane + 64u * it, kc = k < NQ ? k : NQ - 1u;
            const uint32_t r0 = 4u * kc / OD, r1 = (4u * kc + 3u) / OD;
            const bool s0 = (mask >> r0) & 1ull, s1 = (mask >> r1) & 1ull;
            on[it] = k < NQ && (s0 || s1) == dirty;
            if (!dirty) {
                v[it] = a4[kc];                  // clean chunks: no row of theirs reset
            } else {
                // a dirty chunk straddling a reset and a non-reset row is merged from both
                const f4x x = a4[kc], y = b4[kc];
                const uint32_t cut = r1 * OD - 4u * kc;        // first component of row r1
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) v[it][j] = (j >= cut ? s1 : s0) ? y[j] : x[j];
            }
        }
#pragma unroll
        for (uint32_t it = 0; it < IT; ++it)
            if (on[it]) __builtin_nontemporal_store(v[it], dst4 + lane + 64u * it);
    } else {
        const f2x* a2 = reinterpret_cast<const f2x*>(s_obs);
        const f2x* b2 = reinterpret_cast<const f2x*>(s_rrow);
        f2x* dst2 = reinterpret_cast<f2x*>(dst);
        for (uint32_t k = lane; k < nvalid * OD / 2; k += 64u) {
            const bool sr = (mask >> ((2u * k) / OD)) & 1ull;      // OD is even: a pair never spans rows
            if (sr != dirty) continue;
            __builtin_nontemporal_store((sr ? b2 : a2)[k], dst2 + k);
        }
    }
}

// ------------------------------------------------------------------------------------
// per-env register state
// ------------------------------------------------------------------------------------
struct Env {
    float p[3], q[4], v[3], w[3];   // w: world angular velocity (bullet) / body rates (simple)
    float rpy[3], wb[3];            // derived readback (drone.rpy, drone.rpy_dot)
    float x[4], xl[4], ou[4], abuf[4][4];   // motor state x + xl (compensated pair)
    float bias[3], lpf[3], held[10];
    float obs_prev[17];
    float hact[2][4];
    float dt, m, J[3], k0, k1, B[4], K[4];
    float dstb[3], level;
    int ep_step, aidx, halias0, halias1, la_view, props_on, level_idx, gust_left;
    uint32_t rng;
    float la[4];                    // drone.last_action
};

// ------------------------------------------------------------------------------------
// State access: AoSoA float4 groups through a buffer descriptor (cf2sim_internal.h, "internal
// state layout").  One VGPR offset (tile base + lane * 16) serves every group; the group
// offset g * 1024 is a constant the backend splits into the instruction's immediate offset
// and a shared SGPR.  Every access is one coalesced dwordx4 per lane (1 KB per wave).
// ------------------------------------------------------------------------------------
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
struct F4 { float x, y, z, w; };
__device__ __forceinline__ F4 f4(float x, float y, float z, float w) { return F4{x, y, z, w}; }
__device__ __forceinline__ float ib(int v) { return __int_as_float(v); }       // int field -> slot bits
__device__ __forceinline__ int bi(float v) { return __float_as_int(v); }

// ST_AUX: cache-policy bits of the state stores.  2 = nt: the step kernel's stores when the
// working set exceeds the Infinity Cache (launch_step_t) -- at 1 Mi envs 185 -> 144 us, while at
// 262 144 envs (cache-resident) nt stores cost +3 us, as nt loads do at both sizes (the loads
// always use the default policy).
template <int ST_AUX = 0>
struct TileT {
    __amdgpu_buffer_rsrc_t r;
    uint32_t voff;
    __device__ __forceinline__ TileT(const void* base, uint32_t N, uint32_t i)
        : r(__builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)(uint32_t)state_bytes(N), 0x00020000)),
          voff((i >> 6) * (uint32_t)(NG * 1024) + (i & 63u) * 16u) {}
    __device__ __forceinline__ F4 ld(int g) const {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(voff + (uint32_t)g * 1024u), 0, 0);
        return F4{__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w)};
    }
    __device__ __forceinline__ void st(int g, F4 f) const {
        const u32x4 v = {__float_as_uint(f.x), __float_as_uint(f.y), __float_as_uint(f.z), __float_as_uint(f.w)};
        __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)(voff + (uint32_t)g * 1024u), 0, ST_AUX);
    }
};
using Tile = TileT<>;

// G_LPF: with sensor noise the gyro LPF state shares the last o_{k-1} group (13 of its 16 slots
// are o_{k-1}): that group is read with the state, the other three with the history
enum : int { G_CORE3 = 3, G_MOTOR = 4, G_OU = 5, G_ABUF = 6, G_BIAS = 10, G_LPF = 19, G_RPY = 12, G_DSTB = 13,
             G_HACT = 14, G_OBSP = 16, G_HELD = 21, G_PARAM = 24, G_LEVEL = 27, G_MOTOR_LO = 28,
             G_LEVEL_IDX = 29 };

__device__ __forceinline__ bool gust_mode(const KParams& P) { return P.dstb_mode == DSTB_GUST_T; }
__device__ __forceinline__ bool dstb_stored(const KParams& P) {
    return P.dstb_mode == DSTB_CONST_T || P.dstb_mode == DSTB_GUST_T;
}

template <bool NOISE>
__device__ __forceinline__ void load_hist(const Tile& T, Env& E) {
    constexpr int OL = NOISE ? 13 : 17;
    const F4 h0 = T.ld(G_HACT), h1 = T.ld(G_HACT + 1);
    E.hact[0][0] = h0.x; E.hact[0][1] = h0.y; E.hact[0][2] = h0.z; E.hact[0][3] = h0.w;
    E.hact[1][0] = h1.x; E.hact[1][1] = h1.y; E.hact[1][2] = h1.z; E.hact[1][3] = h1.w;
#pragma unroll
    for (int g = 0; g < (NOISE ? 3 : (OL + 3) / 4); ++g) {     // noise: o_{k-1}[12] came with the LPF
        const F4 o = T.ld(G_OBSP + g);
        const float v[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (4 * g + k < OL) E.obs_prev[4 * g + k] = v[k];
    }
}

template <bool NOISE, bool DR, int PHYS>
__device__ __forceinline__ void load_env(const KParams& P, const float* __restrict__ sf, uint32_t i, Env& E,
                                         bool need_level = true, bool with_hist = true) {
    const Tile T(sf, P.N, i);
    const F4 g0 = T.ld(0), g1 = T.ld(1), g2 = T.ld(2), g3 = T.ld(3), gx = T.ld(G_MOTOR), go = T.ld(G_OU);
    E.p[0] = g0.x; E.p[1] = g0.y; E.p[2] = g0.z; E.q[0] = g0.w;
    E.q[1] = g1.x; E.q[2] = g1.y; E.q[3] = g1.z; E.v[0] = g1.w;
    E.v[1] = g2.x; E.v[2] = g2.y; E.w[0] = g2.z; E.w[1] = g2.w;
    E.w[2] = g3.x;
    E.ep_step = bi(g3.y);
    E.rng = (uint32_t)bi(g3.z);
    const int fl = bi(g3.w);
    E.aidx = fl & 15; E.halias0 = (fl >> 4) & 1; E.halias1 = (fl >> 5) & 1; E.la_view = (fl >> 6) & 1;
    E.props_on = (fl >> 7) & 1;
    E.x[0] = gx.x; E.x[1] = gx.y; E.x[2] = gx.z; E.x[3] = gx.w;
    {
        F4 xl = f4(0.0f, 0.0f, 0.0f, 0.0f);
        if (P.use_motor_dyn) xl = T.ld(G_MOTOR_LO);
        E.xl[0] = xl.x; E.xl[1] = xl.y; E.xl[2] = xl.z; E.xl[3] = xl.w;
    }
    E.ou[0] = go.x; E.ou[1] = go.y; E.ou[2] = go.z; E.ou[3] = go.w;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        F4 a = f4(0.0f, 0.0f, 0.0f, 0.0f);
        if (r < P.buf_size) a = T.ld(G_ABUF + r);
        E.abuf[r][0] = a.x; E.abuf[r][1] = a.y; E.abuf[r][2] = a.z; E.abuf[r][3] = a.w;
    }
    E.gust_left = 0;
    if (NOISE || gust_mode(P)) {
        const F4 b = T.ld(G_BIAS);
        if (NOISE) { E.bias[0] = b.x; E.bias[1] = b.y; E.bias[2] = b.z; }
        if (gust_mode(P)) E.gust_left = bi(b.w);
    }
    if (NOISE) {
        const F4 l = T.ld(G_LPF);
        E.obs_prev[12] = l.x; E.lpf[0] = l.y; E.lpf[1] = l.z; E.lpf[2] = l.w;
#pragma unroll
        for (int k = 0; k < 10; ++k) E.held[k] = 0.0f;
        if (P.held_persistent) {
            const F4 h0 = T.ld(G_HELD), h1 = T.ld(G_HELD + 1), h2 = T.ld(G_HELD + 2);
            const float hv[12] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w, h2.x, h2.y, h2.z, h2.w};
#pragma unroll
            for (int k = 0; k < 10; ++k) E.held[k] = hv[k];
        }
    }
    if (PHYS == PHYS_SIMPLE_T) {
        const F4 r = T.ld(G_RPY);
        E.rpy[0] = r.x; E.rpy[1] = r.y; E.rpy[2] = r.z;
    }
    if (dstb_stored(P)) {
        const F4 d = T.ld(G_DSTB);
        E.dstb[0] = d.x; E.dstb[1] = d.y; E.dstb[2] = d.z;
    } else {
        E.dstb[0] = E.dstb[1] = E.dstb[2] = 0.0f;
    }
    if (with_hist) load_hist<NOISE>(T, E);
    F4 lv = f4(0.0f, 0.0f, 0.0f, P.level_fixed);
    if (DR) {
        const F4 p0 = T.ld(G_PARAM), p1 = T.ld(G_PARAM + 1), p2 = T.ld(G_PARAM + 2);
        lv = T.ld(G_LEVEL);
        E.dt = p0.x; E.m = p0.y; E.J[0] = p0.z; E.J[1] = p0.w;
        E.J[2] = p1.x; E.k0 = p1.y; E.k1 = p1.z; E.B[0] = p1.w;
        E.B[1] = p2.x; E.B[2] = p2.y; E.B[3] = p2.z; E.K[0] = p2.w;
        E.K[1] = lv.x; E.K[2] = lv.y; E.K[3] = lv.z;
    } else {
        E.dt = P.time_step; E.m = P.mass; E.J[0] = P.ixx; E.J[1] = P.iyy; E.J[2] = P.izz;
        E.k0 = P.ft0; E.k1 = P.ft1;
#pragma unroll
        for (int k = 0; k < 4; ++k) { E.B[k] = P.B; E.K[k] = P.K; }
        if (need_level) lv = T.ld(G_LEVEL);
    }
    E.level = need_level ? lv.w : P.level_fixed;
    // the level index only matters where levels are redrawn (Boltzmann: the HJ table and the
    // reset keep it); a fixed-level env's index is 0 and its group is not read
    E.level_idx = need_level && P.level_mode != LEVEL_FIXED_T ? bi(T.ld(G_LEVEL_IDX).x) : 0;
}

// state the physics sub-steps update (stored as soon as the last sub-step is done; group 3,
// which carries the counters, is stored with the history at the end of the step)
template <bool NOISE, bool DR, int PHYS, int ST_AUX = 0>
__device__ __forceinline__ void store_core(const KParams& P, float* __restrict__ sf, uint32_t i, const Env& E) {
    const TileT<ST_AUX> T(sf, P.N, i);
    T.st(0, f4(E.p[0], E.p[1], E.p[2], E.q[0]));
    T.st(1, f4(E.q[1], E.q[2], E.q[3], E.v[0]));
    T.st(2, f4(E.v[1], E.v[2], E.w[0], E.w[1]));
    T.st(G_MOTOR, f4(E.x[0], E.x[1], E.x[2], E.x[3]));
    if (P.use_motor_dyn) T.st(G_MOTOR_LO, f4(E.xl[0], E.xl[1], E.xl[2], E.xl[3]));
    T.st(G_OU, f4(E.ou[0], E.ou[1], E.ou[2], E.ou[3]));
#pragma unroll
    for (int r = 0; r < 4; ++r)
        if (r < P.buf_size) T.st(G_ABUF + r, f4(E.abuf[r][0], E.abuf[r][1], E.abuf[r][2], E.abuf[r][3]));
    if (NOISE || gust_mode(P))
        T.st(G_BIAS, f4(NOISE ? E.bias[0] : 0.0f, NOISE ? E.bias[1] : 0.0f, NOISE ? E.bias[2] : 0.0f, ib(E.gust_left)));
    if (NOISE && P.held_persistent) {      // (the LPF state is stored with the history, store_tail)
        T.st(G_HELD, f4(E.held[0], E.held[1], E.held[2], E.held[3]));
        T.st(G_HELD + 1, f4(E.held[4], E.held[5], E.held[6], E.held[7]));
        T.st(G_HELD + 2, f4(E.held[8], E.held[9], 0.0f, 0.0f));
    }
    if (PHYS == PHYS_SIMPLE_T) T.st(G_RPY, f4(E.rpy[0], E.rpy[1], E.rpy[2], 0.0f));
    if (gust_mode(P)) T.st(G_DSTB, f4(E.dstb[0], E.dstb[1], E.dstb[2], 0.0f));
}

// the o_{k-1} groups; with sensor noise the last one carries the gyro LPF state
template <bool NOISE, class TT>
__device__ __forceinline__ void store_obs_prev(const TT& T, const Env& E) {
    constexpr int OL = NOISE ? 13 : 17;
#pragma unroll
    for (int g = 0; g < (OL + 3) / 4; ++g) {
        float v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = 4 * g + k < OL ? E.obs_prev[4 * g + k] : 0.0f;
        if (NOISE && G_OBSP + g == G_LPF) { v[1] = E.lpf[0]; v[2] = E.lpf[1]; v[3] = E.lpf[2]; }
        T.st(G_OBSP + g, f4(v[0], v[1], v[2], v[3]));
    }
}

// end of the step: history, counters (group 3 with the last angular-rate component)
template <bool NOISE, int ST_AUX = 0>
__device__ __forceinline__ void store_tail(const KParams& P, float* __restrict__ sf, uint32_t i, const Env& E) {
    const TileT<ST_AUX> T(sf, P.N, i);
    T.st(G_HACT, f4(E.hact[0][0], E.hact[0][1], E.hact[0][2], E.hact[0][3]));
    T.st(G_HACT + 1, f4(E.hact[1][0], E.hact[1][1], E.hact[1][2], E.hact[1][3]));
    store_obs_prev<NOISE>(T, E);
    const int fl = (E.aidx & 15) | (E.halias0 << 4) | (E.halias1 << 5) | (E.la_view << 6) | (E.props_on << 7);
    T.st(G_CORE3, f4(E.w[2], ib(E.ep_step), ib((int)E.rng), ib(fl)));
}

// whole state (reset paths): core + history + per-episode parameters + counters
template <bool NOISE, bool DR, int PHYS>
__device__ __forceinline__ void store_env(const KParams& P, float* __restrict__ sf, uint32_t i, const Env& E,
                                          bool params_dirty) {
    const Tile T(sf, P.N, i);
    store_core<NOISE, DR, PHYS>(P, sf, i, E);
    store_tail<NOISE>(P, sf, i, E);
    if (P.dstb_mode == DSTB_CONST_T && params_dirty) T.st(G_DSTB, f4(E.dstb[0], E.dstb[1], E.dstb[2], 0.0f));
    if (params_dirty) {
        if (DR) {
            T.st(G_PARAM, f4(E.dt, E.m, E.J[0], E.J[1]));
            T.st(G_PARAM + 1, f4(E.J[2], E.k0, E.k1, E.B[0]));
            T.st(G_PARAM + 2, f4(E.B[1], E.B[2], E.B[3], E.K[0]));
        }
        T.st(G_LEVEL, f4(E.K[1], E.K[2], E.K[3], E.level));
        T.st(G_LEVEL_IDX, f4(ib(E.level_idx), 0.0f, 0.0f, 0.0f));
    }
}

// ------------------------------------------------------------------------------------
// physics
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void apply_action(const KParams& P, Env& E, const float a[4], const float on[4],
                                             float f[4], float& tz) {
    float pwm[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) E.la[j] = a[j];
    E.la_view = 0;
    if (P.use_latency) {
        float del[4];
        // dynamic ring index resolved with selects (no scratch)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float d = opaque(E.abuf[0][j]);
#pragma unroll
            for (int r = 1; r < 4; ++r) d = E.aidx == r ? opaque(E.abuf[r][j]) : d;
            del[j] = d;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < 4; ++j) E.abuf[r][j] = E.aidx == r ? a[j] : E.abuf[r][j];
        E.aidx = E.aidx + 1 == P.buf_size ? 0 : E.aidx + 1;
#pragma unroll
        for (int j = 0; j < 4; ++j) pwm[j] = 30000.0f + clampf(del[j], -1.0f, 1.0f) * 30000.0f;
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) pwm[j] = 30000.0f + clampf(a[j], -1.0f, 1.0f) * 30000.0f;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float xo = E.ou[j];
        const float dx = 0.15f * (0.0f - xo) + P.ou_sigma * on[j];
        E.ou[j] = xo + dx;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float tn = pwm[j] * (1.0f / 60000.0f);      // == pwm / 60000 as compiled (see DIV_NOTE)
        float noisy;
        if (P.use_motor_dyn) {
            // x(k+1) = A x(k) + B u with A = 1 - B (agents.py:288), evaluated as x += B (u - x) on the
            // unevaluated pair x + xl (TwoSum): the recurrence then carries no fp32 rounding from
            // step to step (it dominated the drift vs the fp64 reference)
            const float rot = sqrt_fast(tn);
            const float inc = E.B[j] * ((rot - E.x[j]) - E.xl[j]);
            const float sum = E.x[j] + inc, bb = sum - E.x[j];                  // TwoSum
            const float lo = ((E.x[j] - (sum - bb)) + (inc - bb)) + E.xl[j];
            E.x[j] = sum + lo;                                                    // renormalise
            E.xl[j] = lo - (E.x[j] - sum);
            noisy = (1.0f + E.ou[j]) * (E.x[j] * E.x[j]);
        } else {
            noisy = (1.0f + E.ou[j]) * tn;
        }
        // rounded on its own (no FMA contraction into the mixer sums below): equal motor forces then
        // cancel exactly in the roll/pitch torques, as in the reference; a contracted product would
        // leave a one-sided ulp torque every sub-step (a systematic attitude drift in hover)
        f[j] = opaque(E.K[j] * clampf(noisy, 0.0f, 1.0f));
    }
    float t[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) t[j] = E.k1 * f[j] + E.k0;
    tz = (-t[0] + t[1] - t[2] + t[3]);
}

// GE: calculate_ground_effect on (physics_kernel only: the reference's envs never enable it, and the
// env-step kernels keep their code free of the branch)
template <bool GE = false>
__device__ __forceinline__ void bullet_substep(const KParams& P, Env& E, const float a[4], const float d[3],
                                               const float on[4], bool first_after_reset, float dw = 0.0f) {
    float xprev[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) xprev[j] = E.x[j];
    float f[4], tz;
    apply_action(P, E, a, on, f, tz);
    const M3 R = rotmat(E.q);
    float ssum = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float rpm = E.x[j] * E.x[j] * 25000.0f;
        ssum += 2.0f * 3.141592653589793f * rpm * (1.0f / 60.0f);     // DIV_NOTE
    }
    const float dl[3] = {-1.0f * P.drag_xy * ssum * E.v[0], -1.0f * P.drag_xy * ssum * E.v[1], -1.0f * P.drag_z * ssum * E.v[2]};
    float drag1[3], dragw[3];
    mv(R, dl, drag1);
    mv(R, drag1, dragw);
    const float L = P.prop_xy;
    const float mp = P.prop_mass, Ip = P.prop_inertia, Lz = P.prop_z;
    if (GE && fabsf(E.rpy[0]) < 1.5707963267948966f && fabsf(E.rpy[1]) < 1.5707963267948966f) {
        // BasePhysics.calculate_ground_effect (physics.py:27-58): extra thrust at each prop from its
        // height z_i = (p + R o_i)_z (getLinkStates), clipped at GND_EFF_H_CLIP; added to the prop
        // forces (apply_motor_forces, physics.py:243-246), not to the yaw torque.  rpy: the last readback.
        const float ox[4] = {L, -L, -L, L}, oy[4] = {-L, -L, L, L};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float z = fmaxf(E.p[2] + (R.m[6] * ox[j] + R.m[7] * oy[j] + R.m[8] * Lz), P.gnd_eff_h_clip);
            const float rr = P.prop_radius * rcp(4.0f * z);
            f[j] = opaque(f[j] + f[j] * P.gnd_eff_coeff * (rr * rr));
        }
    }
    float tb[3];
    tb[0] = L * (-f[0] - f[1] + f[2] + f[3]) + d[0];
    tb[1] = L * (-f[0] + f[1] + f[2] - f[3]) + d[1];
    tb[2] = tz;
    const float fsum = f[0] + f[1] + f[2] + f[3];
    const float mtot = E.m + 4.0f * mp;
    float Fw[3];
    const float fz = fsum - dw;      // downwash of formation mates: -z of the body, at the COM
    Fw[0] = R.m[2] * fz + dragw[0];
    Fw[1] = R.m[5] * fz + dragw[1];
    Fw[2] = R.m[8] * fz + dragw[2] - P.g_world * mtot;
    float wb[3], vb[3];
    mtv(R, E.w, wb);
    mtv(R, E.v, vb);
    const float wn = norm3(wb), vn = norm3(vb);
    float Ic[3];
    Ic[0] = E.J[0] + 4.0f * Ip + 4.0f * mp * (L * L + Lz * Lz);
    Ic[1] = E.J[1] + 4.0f * Ip + 4.0f * mp * (L * L + Lz * Lz);
    Ic[2] = E.J[2] + 4.0f * Ip + 4.0f * mp * (L * L + L * L);
    const float kq = P.prop_speed_gain;
    const float sp_old = first_after_reset ? 0.0f : kq * (-xprev[0] + xprev[1] - xprev[2] + xprev[3]);
    const float sp_new = kq * (-E.x[0] + E.x[1] - E.x[2] + E.x[3]);
    const float h_old = Ip * sp_old;
    const float Iw[3] = {Ic[0] * wb[0], Ic[1] * wb[1], Ic[2] * wb[2] + h_old};
    const float gyro[3] = {wb[1] * Iw[2] - wb[2] * Iw[1], wb[2] * Iw[0] - wb[0] * Iw[2], wb[0] * Iw[1] - wb[1] * Iw[0]};
    const float dampa = P.ang_damping * (1.0f + wn);
    const float tdamp[3] = {E.J[0] * wb[0] * dampa, E.J[1] * wb[1] * dampa, E.J[2] * wb[2] * dampa};
    float pd[3] = {0.0f, 0.0f, 0.0f};
    {
        const float ax[4] = {-1.0f, 1.0f, -1.0f, 1.0f};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float qd = first_after_reset ? 0.0f : kq * xprev[j];
            const float wp[3] = {wb[0], wb[1], wb[2] + ax[j] * qd};
            const float k = Ip * P.ang_damping * (1.0f + norm3(wp));
            pd[0] += k * wp[0]; pd[1] += k * wp[1]; pd[2] += k * wp[2];
        }
    }
    const float dt = E.dt;
    float wdot_b[3];
    wdot_b[0] = (tb[0] - gyro[0] - tdamp[0] - pd[0]) * rcp(Ic[0]);
    wdot_b[1] = (tb[1] - gyro[1] - tdamp[1] - pd[1]) * rcp(Ic[1]);
    wdot_b[2] = (tb[2] - gyro[2] - tdamp[2] - pd[2] - Ip * (sp_new - sp_old) * rcp(dt)) * rcp(Ic[2]);
    const float imtot = rcp(mtot);
    const float dampl = P.lin_damping * (1.0f + vn) * E.m * imtot;
    float vdot_w[3], wdot_w[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) vdot_w[k] = Fw[k] * imtot - dampl * E.v[k];
    mv(R, wdot_b, wdot_w);
    const float vmax = P.vmax;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        E.w[k] = clampf(E.w[k] + wdot_w[k] * dt, -vmax, vmax);
        E.v[k] = clampf(E.v[k] + vdot_w[k] * dt, -vmax, vmax);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) E.p[k] += dt * E.v[k];
    {
        float ang = norm3(E.w);
        ang = ang * dt > 0.7853981633974483f ? 0.7853981633974483f * rcp(dt) : ang;
        // half-angle h = ang*dt/2 <= pi/8 after the clamp: odd/even Taylor polynomials are exact to
        // fp32 there (truncation < 3e-13), cheaper and more accurate than the hardware sin/cos
        const float h = 0.5f * ang * dt, h2 = h * h;
        const float sin_h = h * (1.0f + h2 * (-1.6666667e-1f + h2 * (8.3333333e-3f + h2 * (-1.9841270e-4f + h2 * 2.7557319e-6f))));
        const float cw = 1.0f + h2 * (-0.5f + h2 * (4.1666668e-2f + h2 * (-1.3888889e-3f + h2 * (2.4801587e-5f - h2 * 2.7557319e-7f))));
        const float s = ang < 0.001f ? 0.5f * dt - (dt * dt * dt) * 0.020833333333f * ang * ang : sin_h * rcp(ang);
        const float axs[3] = {E.w[0] * s, E.w[1] * s, E.w[2] * s};
        const float qx = E.q[0], qy = E.q[1], qz = E.q[2], qw = E.q[3];
        const float nx = cw * qx + axs[0] * qw + axs[1] * qz - axs[2] * qy;
        const float ny = cw * qy + axs[1] * qw + axs[2] * qx - axs[0] * qz;
        const float nz = cw * qz + axs[2] * qw + axs[0] * qy - axs[1] * qx;
        const float nw = cw * qw - axs[0] * qx - axs[1] * qy - axs[2] * qz;
        const float il = rsq(nx * nx + ny * ny + nz * nz + nw * nw);
        E.q[0] = nx * il; E.q[1] = ny * il; E.q[2] = nz * il; E.q[3] = nw * il;
    }
    // update_information
    euler_from_quat(E.q, E.rpy);
    const M3 Rn = rotmat(E.q);
    mtv(Rn, E.w, E.wb);
}

__device__ __forceinline__ void simple_substep(const KParams& P, Env& E, const float a[4], const float on[4]) {
    float f[4], tz;
    apply_action(P, E, a, on, f, tz);
    const M3 R = rotmat(E.q);
    const float fsum = f[0] + f[1] + f[2] + f[3];
    const float Fw[3] = {R.m[2] * fsum - 0.0f * E.m, R.m[5] * fsum - 0.0f * E.m, R.m[8] * fsum - P.g_world * E.m};
    const float tx = (-f[0] - f[1] + f[2] + f[3]) * P.arm / sqrtf(2.0f);
    const float ty = (-f[0] + f[1] + f[2] - f[3]) * P.arm / sqrtf(2.0f);
    float* w = E.wb;
    const float Jw[3] = {E.J[0] * w[0], E.J[1] * w[1], E.J[2] * w[2]};
    const float cr[3] = {w[1] * Jw[2] - w[2] * Jw[1], w[2] * Jw[0] - w[0] * Jw[2], w[0] * Jw[1] - w[1] * Jw[0]};
    const float t[3] = {tx - cr[0], ty - cr[1], tz - cr[2]};
    const float wdd[3] = {rcp(E.J[0]) * t[0], rcp(E.J[1]) * t[1], rcp(E.J[2]) * t[2]};
    const float im = rcp(E.m);
    const float acc[3] = {Fw[0] * im, Fw[1] * im, Fw[2] * im};
    const float dt = E.dt;
#pragma unroll
    for (int k = 0; k < 3; ++k) E.v[k] += dt * acc[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) E.wb[k] += dt * wdd[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) E.p[k] += dt * E.v[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) E.rpy[k] += dt * E.wb[k];
    quat_from_euler(E.rpy, E.q);
    if (E.p[2] < 0.0f) E.p[2] = 0.0f;
#pragma unroll
    for (int k = 0; k < 3; ++k) E.w[k] = E.wb[k];   // simple mode stores body rates in F_OMEGA
}

// ------------------------------------------------------------------------------------
// observation / history / reward
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void omega_noise(const KParams& P, Env& E, const float* n, float om[3]) {
#pragma unroll
    for (int k = 0; k < 3; ++k) E.bias[k] = P.pgd * E.bias[k] + P.sbgd * n[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) om[k] = E.wb[k] + E.bias[k] + P.gyro_rw * n[3 + k] + P.gyro_ton * n[6 + k];
}

// A full measurement's held part (noisy position, attitude quaternion and velocity,
// sensors.py:75-118) and its 9 gyro normals n[6..15) (bias walk, white noise, turn-on noise): what
// the measurement draws from stream blocks base..base+5.  The gyro part is applied by
// gyro_update, which needs the body rates, bias and LPF state of the moment.  Split in two so the
// draws can run before the state they perturb is known (the small-N kernel's helper waves):
// held_noise turns the draws into the position / velocity / rpy perturbations, held_combine adds
// them.  The velocity perturbation is rounded on its own (no fma into the sum), as the fp32
// restatement computes v + vel_std * n.
struct HeldNoise { float pn[3], vn[3], th[3]; };
template <class G>
__device__ __forceinline__ void held_noise(const KParams& P, const G& g, uint32_t base, HeldNoise& h, float ng[9]) {
    float n[18];
    normals<18>(g, base, n);
    const U4 ua = g.block(base + 4), ub = g.block(base + 5);
    const uint32_t up[3] = {ua.z, ua.w, ub.x}, ur[3] = {ub.y, ub.z, ub.w};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float uo = -P.pos_unif + (P.pos_unif - -P.pos_unif) * u01(up[k]);
        h.pn[k] = P.pos_std * n[k] + uo;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) h.vn[k] = opaque(P.vel_std * n[3 + k]);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float uo = -P.rot_unif + (P.rot_unif - -P.rot_unif) * u01(ur[k]);
        h.th[k] = P.rot_std * n[15 + k] + uo;
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) ng[k] = n[6 + k];
}
__device__ __forceinline__ void held_combine(const Env& E, const HeldNoise& h, float held[10]) {
#pragma unroll
    for (int k = 0; k < 3; ++k) held[k] = E.p[k] + h.pn[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) held[7 + k] = E.v[k] + h.vn[k] + 0.0f;
    const float lo[3] = {-3.141592653589793f, -1.5707963267948966f, -3.141592653589793f};
    float rot[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) rot[k] = clampf(E.rpy[k] + h.th[k], lo[k], -lo[k]);
    quat_from_euler_obs(rot, held + 3);
}
template <class G>
__device__ __forceinline__ void held_measurement(const KParams& P, const Env& E, const G& g, uint32_t base,
                                                 float held[10], float ng[9]) {
    HeldNoise h;
    held_noise(P, g, base, h, ng);
    held_combine(E, h, held);
}

// gyro of one sensor call: bias walk + noise on the body rates, then the gyro low-pass filter
// (sensors.py:121-134, utils.py:102-105); ng = the call's 9 gyro normals
__device__ __forceinline__ void gyro_update(const KParams& P, Env& E, const float ng[9]) {
    float om[3];
    omega_noise(P, E, ng, om);
#pragma unroll
    for (int k = 0; k < 3; ++k) E.lpf[k] = (1.0f - P.lpf_ratio) * E.lpf[k] + P.lpf_gain * P.lpf_ratio * om[k];
}

// need_held = false: the held measurement of this call is dead (it is overwritten by a later
// full measurement before any observation is emitted), so a full measurement only advances the
// gyro (bias walk + LPF) and draws just the gyro normals n[6..15) of its stream positions.
template <bool NOISE, class G>
__device__ __forceinline__ void compute_observation(const KParams& P, Env& E, const G& g, uint32_t base,
                                                    int iteration, float* obs, bool need_held = true) {
    if (!NOISE) {
#pragma unroll
        for (int k = 0; k < 3; ++k) obs[k] = E.p[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) obs[3 + k] = E.q[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) obs[7 + k] = E.v[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) obs[10 + k] = E.wb[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) obs[13 + k] = E.la[k];
        return;
    }
    const bool full = (uint32_t)iteration % (uint32_t)P.obs_rate == 0u;
    if (full && !need_held) {
        float n[18];
        normals_range<6, 15>(g, base, n);
        gyro_update(P, E, n + 6);
    } else if (full) {
        float held[10], ng[9];
        held_measurement(P, E, g, base, held, ng);
        gyro_update(P, E, ng);
#pragma unroll
        for (int k = 0; k < 10; ++k) E.held[k] = held[k];
    } else {
        float n[9];
        normals<9>(g, base, n);
        gyro_update(P, E, n);
    }
#pragma unroll
    for (int k = 0; k < 10; ++k) obs[k] = E.held[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) obs[10 + k] = E.lpf[k];
}

__device__ __forceinline__ bool compute_done(const KParams& P, const Env& E) {
    const bool rp = fabsf(E.rpy[0]) > P.done_rp || fabsf(E.rpy[1]) > P.done_rp;
    bool rt = false;
#pragma unroll
    for (int k = 0; k < 3; ++k) rt |= (180.0f * fabsf(E.wb[k]) * (1.0f / 3.141592653589793f)) > P.done_rate_deg;   // DIV_NOTE
    return rp || rt || (E.p[2] < P.done_zmin);
}

__device__ __forceinline__ float compute_reward(const KParams& P, const Env& E, const float a[4], bool done) {
    float na[4], ad[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) { na[k] = 0.5f * (clampf(a[k], -1.0f, 1.0f) + 1.0f); ad[k] = a[k] - E.la[k]; }
    const float nna = sqrt_fast(na[0] * na[0] + na[1] * na[1] + na[2] * na[2] + na[3] * na[3]);
    const float nad = sqrt_fast(ad[0] * ad[0] + ad[1] * ad[1] + ad[2] * ad[2] + ad[3] * ad[3]);
    float dr[3], dw[3], dp[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        dr[k] = E.rpy[k] - P.target_rpy[k];
        dw[k] = E.wb[k] - P.target_rate[k];
        dp[k] = E.p[k] - P.target_pos[k];
    }
    float pen = 0.0f;
    pen += P.pen_angle * norm3(dr);
    pen += P.pen_arp * nad;
    pen += P.pen_spin * norm3(dw);
    pen += P.pen_vel * norm3(E.v);
    pen += P.pen_action * nna;
    pen += done ? P.pen_term : 0.0f;
    const float zd = P.pen_z * fabsf(E.p[2] - P.target_pos[2]);
    const float dist = P.pen_dist * norm3(dp);
    return -pen - zd - dist;
}

__device__ __forceinline__ float compute_cost(const KParams& P, const Env& E) {
    float c = 0.0f;
    if (fabsf(E.p[0]) > P.cost_xy || fabsf(E.p[1]) > P.cost_xy || E.p[2] > P.cost_z) c = 1.0f;
    if (fabsf(E.rpy[0]) > P.cost_rp || fabsf(E.rpy[1]) > P.cost_rp) c = 1.0f;
#pragma unroll
    for (int k = 0; k < 3; ++k) if (fabsf(E.wb[k]) > P.cost_vel) c = 1.0f;
#pragma unroll
    for (int k = 0; k < 3; ++k) if (fabsf(E.la[k]) > P.cost_rate) c = 1.0f;
    return c;
}

__device__ __forceinline__ void abuf_last(const KParams& P, const Env& E, float o[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        float v = opaque(E.abuf[0][j]);
#pragma unroll
        for (int r = 1; r < 4; ++r) v = (P.buf_size - 1) == r ? opaque(E.abuf[r][j]) : v;
        o[j] = v;
    }
}

// compute_history: writes out[obs_dim] = [obs_prev, A0, obs_next, A1]
template <bool NOISE>
__device__ __forceinline__ void compute_history(const KParams& P, Env& E, const float* on, float* out) {
    constexpr int OL = NOISE ? 13 : 17;
    float last[4];
    abuf_last(P, E, last);
    int o = 0;
#pragma unroll
    for (int k = 0; k < OL; ++k) out[o++] = E.obs_prev[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) out[o++] = E.halias0 ? last[k] : E.hact[0][k];
#pragma unroll
    for (int k = 0; k < OL; ++k) out[o++] = on[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) out[o++] = E.halias1 ? last[k] : E.hact[1][k];
#pragma unroll
    for (int k = 0; k < OL; ++k) E.obs_prev[k] = on[k];
    E.halias0 = E.halias1;
#pragma unroll
    for (int k = 0; k < 4; ++k) E.hact[0][k] = E.hact[1][k];
    E.halias1 = E.la_view;
#pragma unroll
    for (int k = 0; k < 4; ++k) E.hact[1][k] = E.la[k];
}

__device__ __forceinline__ int boltzmann_index(const KParams& P, float u) {
    int i = 0;
    for (int k = 0; k < P.num_levels - 1; ++k) i += ((double)u < P.tab->level_cdf[k]) ? 0 : 1;
    // cdf is non-decreasing: count of entries <= u == searchsorted(side='right')
    return i;
}

// ------------------------------------------------------------------------------------
// multi-drone formations (no reference implementation): the drones of a
// group are consecutive lanes of one wave, so mates' positions are wave shuffles
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void formation_offset(const KParams& P, uint32_t member, float off[3]) {
    const int ncol = (P.num_drones + 1) / 2;
    off[0] = P.num_drones > 1 ? ((float)(int)(member / 2) - (float)(ncol - 1) * 0.5f) * P.formation_dx : 0.0f;
    off[1] = 0.0f;
    off[2] = P.num_drones > 1 ? (float)(int)(member % 2) * P.formation_dz : 0.0f;
}
// gym-pybullet-drones BaseAviary._downwash summed over the mates above this drone
__device__ __forceinline__ float downwash(const KParams& P, const float p[3], uint32_t member) {
    float F = 0.0f;
    for (int j = 0; j < P.num_drones; ++j) {
        const float qx = __shfl(p[0], j, P.num_drones), qy = __shfl(p[1], j, P.num_drones),
                    qz = __shfl(p[2], j, P.num_drones);
        const float dz = qz - p[2], dx = qx - p[0], dy = qy - p[1];
        const float dxy = sqrt_fast(dx * dx + dy * dy);
        if ((uint32_t)j != member && dz > 0.0f && dxy < 10.0f) {
            const float rr = P.prop_radius * rcp(4.0f * dz);
            const float alpha = P.dw_coeff[0] * rr * rr;
            const float q = dxy * rcp(P.dw_coeff[1] * dz + P.dw_coeff[2]);
            F += alpha * __builtin_amdgcn_exp2f(-0.72134752044448170f * q * q);   // exp(-q^2/2)
        }
    }
    return F;
}

// The env-step's kernel parameters that only its epilogue reads (done, reward and cost thresholds
// and weights), re-read from the kernarg segment where they are used: every kernel that steps envs
// takes its KParams first, so the segment starts with them.  Through the opaque pointer the loads
// cannot be hoisted to the kernel's entry, where the compiler otherwise issues every kernarg load
// and, with ~100 scalar registers of live values across the physics, spills them to VGPR lanes
// (87 v_writelane / 279 v_readlane sites in the 262 144-env kernel).  The large-N step kernel
// re-reads the epilogue's and the final sensor call's parameters (LATEP) and the auto-reset's
// reset-only ones (reset_src<2>): 24 writelane sites left, 262 144 envs 36.3 -> 33.9 us, HJ
// 41.1 -> 39.6, 65 536 envs 14.7 -> 13.9 (profiles/r06_ab_late_params.txt); the small-N kernel,
// whose spills are few, measured +0.3 us with the epilogue part.
typedef const __attribute__((address_space(4))) KParams* KernargParams;
__device__ __forceinline__ KernargParams kernarg_params() {
    KernargParams p = (KernargParams)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return p;
}
// P with the epilogue's fields re-read (done, reward, cost; the others as in P)
__device__ __forceinline__ KParams late_epilogue(const KParams& P) {
    KParams Q = P;
    const KernargParams k = kernarg_params();
    Q.pen_action = k->pen_action; Q.pen_angle = k->pen_angle; Q.pen_spin = k->pen_spin; Q.pen_term = k->pen_term;
    Q.pen_vel = k->pen_vel; Q.pen_z = k->pen_z; Q.pen_arp = k->pen_arp; Q.pen_dist = k->pen_dist;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        Q.target_pos[j] = k->target_pos[j]; Q.target_rpy[j] = k->target_rpy[j]; Q.target_rate[j] = k->target_rate[j];
    }
    Q.done_rp = k->done_rp; Q.done_rate_deg = k->done_rate_deg; Q.done_zmin = k->done_zmin;
    Q.cost_xy = k->cost_xy; Q.cost_z = k->cost_z; Q.cost_rp = k->cost_rp; Q.cost_vel = k->cost_vel;
    Q.cost_rate = k->cost_rate;
    return Q;
}
// io with the per-env output pointers re-read (StepIO is the second kernel argument of every
// kernel that passes LATEP: step_kernel, collect_kernel)
typedef const __attribute__((address_space(4))) StepIO* KernargIO;
__device__ __forceinline__ StepIO late_outputs(const StepIO& io) {
    constexpr size_t off = (sizeof(KParams) + alignof(StepIO) - 1) / alignof(StepIO) * alignof(StepIO);
    KernargIO k = (KernargIO)((const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr() + off);
    asm volatile("" : "+s"(k));
    StepIO o = io;
    o.rew = k->rew; o.done = k->done; o.trunc = k->trunc; o.cost = k->cost; o.level = k->level;
    o.final_obs = k->final_obs;
    return o;
}
// every pointer of io re-read (the fused rollout derives each env-step's output slabs from them)
__device__ __forceinline__ StepIO late_io(const StepIO& io) {
    constexpr size_t off = (sizeof(KParams) + alignof(StepIO) - 1) / alignof(StepIO) * alignof(StepIO);
    KernargIO k = (KernargIO)((const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr() + off);
    asm volatile("" : "+s"(k));
    StepIO o = io;
    o.sf = k->sf; o.act = k->act; o.dstb = k->dstb; o.obs = k->obs; o.rew = k->rew; o.done = k->done;
    o.trunc = k->trunc; o.cost = k->cost; o.level = k->level; o.final_obs = k->final_obs;
    return o;
}
// P with the physics sub-step's constants re-read (the fused rollout, LATEX: its K-step loop kept
// them live across the whole loop body, spilled with the rest)
__device__ __forceinline__ KParams late_physics(const KParams& P) {
    KParams Q = P;
    const KernargParams k = kernarg_params();
    Q.time_step = k->time_step; Q.mass = k->mass; Q.ixx = k->ixx; Q.iyy = k->iyy; Q.izz = k->izz;
    Q.ft0 = k->ft0; Q.ft1 = k->ft1; Q.K = k->K; Q.B = k->B; Q.ou_sigma = k->ou_sigma;
    Q.drag_xy = k->drag_xy; Q.drag_z = k->drag_z; Q.g_world = k->g_world; Q.arm = k->arm;
    Q.prop_xy = k->prop_xy; Q.prop_z = k->prop_z; Q.prop_mass = k->prop_mass; Q.prop_inertia = k->prop_inertia;
    Q.prop_speed_gain = k->prop_speed_gain; Q.lin_damping = k->lin_damping; Q.ang_damping = k->ang_damping;
    Q.vmax = k->vmax;
    return Q;
}
// P with the reset-only fields re-read (reset_src<2>)
__device__ __forceinline__ KParams late_reset(const KParams& P) {
    KParams Q = P;
    const KernargParams k = kernarg_params();
#pragma unroll
    for (int j = 0; j < 3; ++j) Q.init_xyz[j] = k->init_xyz[j];
    Q.pos_lim = k->pos_lim; Q.angle_lim = k->angle_lim; Q.yaw_lim = k->yaw_lim; Q.vel_lim = k->vel_lim;
    Q.rate_lim = k->rate_lim; Q.yaw_rate_lim = k->yaw_rate_lim; Q.action_std = k->action_std;
    Q.motor_std = k->motor_std; Q.hover_x = k->hover_x; Q.hover_action = k->hover_action;
#pragma unroll
    for (int j = 0; j < 9; ++j) { Q.dr_lo[j] = k->dr_lo[j]; Q.dr_hi[j] = k->dr_hi[j]; }
    return Q;
}

// ------------------------------------------------------------------------------------
// reset (base.py:420-464 + task_specific_reset + apply_domain_randomization)
// ------------------------------------------------------------------------------------
// The reset in three pieces (reset_env runs them in order; the step kernel's auto-reset runs them
// on different waves, see block_epilogue):
//   reset_kinematics  initial pose / velocities (task_specific_reset hover_free.py:237-289), motor
//                     state and latency ring, last action, readback -- what the observation needs;
//   reset_params      domain randomisation (base.py:241-298), const-wind draw, Boltzmann level;
//   reset_observe     the two reset sensor calls (base.py:444-456 incl. the stale-rpy_dot LPF
//                     seed) and the history / observation row.
// where the reset-only parameters are read: TAB 1 = the device tables (P.tab; the fused rollout,
// whose register budget cannot hold them from kernel entry), 2 = the kernarg block re-read at the
// reset (late_reset: the large-N step kernel, where holding them from kernel entry spilled them
// to VGPR lanes), else the kernarg block as loaded at kernel entry
template <int TAB>
__device__ __forceinline__ decltype(auto) reset_src(const KParams& P) {
    if constexpr (TAB == 1) return (*P.tab);
    else if constexpr (TAB == 2) return late_reset(P);
    else return (P);
}

template <int PHYS, int TAB = 0, class G>
__device__ __forceinline__ void reset_kinematics(const KParams& P, Env& E, const G& g, uint32_t gid) {
    const U4 b0 = g.block(0), b1 = g.block(1), b2 = g.block(2), b3 = g.block(3);
    const uint32_t u[16] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w,
                            b2.x, b2.y, b2.z, b2.w, b3.x, b3.y, b3.z, b3.w};
    E.ep_step = 0;
    E.props_on = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) E.x[j] = E.xl[j] = 0.0f;
    E.aidx = 0;
    const auto& Tr = reset_src<TAB>(P);  // reset-only parameters
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j) E.abuf[r][j] = 0.0f;
    float pos[3] = {Tr.init_xyz[0], Tr.init_xyz[1], Tr.init_xyz[2]};
    if (P.num_drones > 1) {
        float off[3];
        formation_offset(P, gid % (uint32_t)P.num_drones, off);
#pragma unroll
        for (int k = 0; k < 3; ++k) pos[k] += off[k];
    }
    float quat[4] = {0.0f, 0.0f, 0.0f, 1.0f};
    float vel[3] = {0.0f, 0.0f, 0.0f}, rate[3] = {0.0f, 0.0f, 0.0f};
    if (P.reset_dist) {
#pragma unroll
        for (int k = 0; k < 3; ++k) pos[k] += -Tr.pos_lim + (Tr.pos_lim - -Tr.pos_lim) * u01(u[k]);
        float rpy[3];
        rpy[0] = -Tr.angle_lim + (Tr.angle_lim - -Tr.angle_lim) * u01(u[4]);
        rpy[1] = -Tr.angle_lim + (Tr.angle_lim - -Tr.angle_lim) * u01(u[5]);
        rpy[2] = -Tr.yaw_lim + (Tr.yaw_lim - -Tr.yaw_lim) * u01(u[3]);
        quat_from_euler(rpy, quat);
#pragma unroll
        for (int k = 0; k < 3; ++k) vel[k] = vel[k] + (-Tr.vel_lim + (Tr.vel_lim - -Tr.vel_lim) * u01(u[8 + k]));
        rate[0] = rate[0] + (-Tr.rate_lim + (Tr.rate_lim - -Tr.rate_lim) * u01(u[11]));
        rate[1] = rate[1] + (-Tr.rate_lim + (Tr.rate_lim - -Tr.rate_lim) * u01(u[12]));
        rate[2] = -Tr.yaw_rate_lim + (Tr.yaw_rate_lim - -Tr.yaw_rate_lim) * u01(u[7]);
        float nx[4];
        normals<4>(g, 4, nx);
#pragma unroll
        for (int j = 0; j < 4; ++j) E.x[j] = Tr.hover_x + Tr.motor_std * nx[j];
        float nb[16];
        normals<16>(g, 5, nb);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                E.abuf[r][j] = r < P.buf_size ? clampf(Tr.hover_action + Tr.action_std * nb[4 * r + j], -1.0f, 1.0f) : 0.0f;
    }
    abuf_last(P, E, E.la);
    E.la_view = 1;
#pragma unroll
    for (int k = 0; k < 3; ++k) { E.p[k] = pos[k]; E.v[k] = vel[k]; }
#pragma unroll
    for (int k = 0; k < 4; ++k) E.q[k] = quat[k];
    const M3 R0 = rotmat(quat);
    float ww[3];
    mtv(R0, rate, ww);
    if (PHYS == PHYS_BULLET_T) {
#pragma unroll
        for (int k = 0; k < 3; ++k) E.w[k] = ww[k];
        euler_from_quat(E.q, E.rpy);
        mtv(R0, E.w, E.wb);      // R(q) of the reset quaternion
    } else {
        euler_from_quat(E.q, E.rpy);
        mtv(R0, ww, E.wb);
#pragma unroll
        for (int k = 0; k < 3; ++k) E.w[k] = E.wb[k];
    }
}

template <bool DR, int TAB = 0, class G>
__device__ __forceinline__ void reset_params(const KParams& P, Env& E, const G& g) {
    E.dt = P.time_step; E.m = P.mass; E.J[0] = P.ixx; E.J[1] = P.iyy; E.J[2] = P.izz;
    E.k0 = P.ft0; E.k1 = P.ft1;
#pragma unroll
    for (int j = 0; j < 4; ++j) { E.B[j] = P.B; E.K[j] = P.K; }
    if (DR) {
        const auto& Tr = reset_src<TAB>(P);   // reset-only parameters
        const U4 d0 = g.block(9), d1 = g.block(10), d2 = g.block(11), d3 = g.block(12);
        const uint32_t d[16] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w,
                                d2.x, d2.y, d2.z, d2.w, d3.x, d3.y, d3.z, d3.w};
#define DRAW(b, ui) (Tr.dr_lo[b] + (Tr.dr_hi[b] - Tr.dr_lo[b]) * u01(d[ui]))
        E.dt = DRAW(0, 0); E.m = DRAW(1, 1);
        E.J[0] = DRAW(2, 2); E.J[1] = DRAW(3, 3); E.J[2] = DRAW(4, 4);
        E.k0 = DRAW(5, 5); E.k1 = DRAW(6, 6);
        if (P.use_motor_dyn) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float mtc = DRAW(7, 7 + j);
                const float t2w = DRAW(8, 11 + j);
                const float T = mtc < E.dt ? E.dt : mtc;
                E.B[j] = E.dt / T;             // A = 1 - B (apply_action's compensated form)
                E.K[j] = 0.028f * P.g_agent * t2w / 4.0f;
            }
        }
#undef DRAW
    }
    {
        const U4 w = g.block(13);
        if (P.dstb_mode == DSTB_CONST_T) {
            const uint32_t wu[3] = {w.x, w.y, w.z};
#pragma unroll
            for (int k = 0; k < 3; ++k) E.dstb[k] = (-1.0f + 2.0f * u01(wu[k])) * P.umax[k] * E.level;
        } else {
#pragma unroll
            for (int k = 0; k < 3; ++k) E.dstb[k] = 0.0f;
        }
        E.gust_left = 0;
    }
    if (P.level_mode == LEVEL_BOLTZMANN_T) {          // the new episode's level (after the const-wind draw)
        E.level_idx = boltzmann_index(P, u01(g.block(3).y));
        E.level = P.tab->level_values[E.level_idx];
    }
}

// stale: the finished episode's body rates (the gyro LPF seed); E.bias is the never-reset gyro bias.
// half: 0 = both calls and the whole observation row; 1 = the first call only, out[0 .. OL+4)
// (o_0 and A_0); 2 = the second call and out[OL+4 .. OD) (o_1, A_1), the first call's gyro walk
// only (its held measurement is not needed there).
template <bool NOISE, int HALF, class G>
__device__ __forceinline__ void reset_observe(const KParams& P, Env& E, const G& g, const float stale[3], float* out) {
    constexpr int OL = NOISE ? 13 : 17;
    if (NOISE) {
#pragma unroll
        for (int k = 0; k < 3; ++k) E.lpf[k] = stale[k];
    }
    float o0[17], o1[17];
    compute_observation<NOISE>(P, E, g, 32, 0, o0, HALF != 2);
#pragma unroll
    for (int k = 0; k < OL; ++k) E.obs_prev[k] = o0[k];
    E.halias0 = E.halias1 = 1;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int k = 0; k < 4; ++k) E.hact[s][k] = E.la[k];
    if (HALF == 1) {
#pragma unroll
        for (int k = 0; k < OL; ++k) out[k] = o0[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) out[OL + k] = E.la[k];      // halias0: the action buffer's last entry
        return;
    }
    compute_observation<NOISE>(P, E, g, 40, 0, o1);
    if (HALF == 2) {
#pragma unroll
        for (int k = 0; k < OL; ++k) { out[OL + 4 + k] = o1[k]; E.obs_prev[k] = o1[k]; }
#pragma unroll
        for (int k = 0; k < 4; ++k) out[2 * OL + 4 + k] = E.la[k];
        E.halias0 = E.halias1;
#pragma unroll
        for (int k = 0; k < 4; ++k) E.hact[0][k] = E.hact[1][k];
        E.halias1 = E.la_view;
#pragma unroll
        for (int k = 0; k < 4; ++k) E.hact[1][k] = E.la[k];
        return;
    }
    compute_history<NOISE>(P, E, o1, out);
}

template <bool NOISE, bool DR, int PHYS, int TAB = 0, class G>
__device__ __forceinline__ void reset_env(const KParams& P, Env& E, const G& g, uint32_t gid, float* out) {
    const float stale[3] = {E.wb[0], E.wb[1], E.wb[2]};
    reset_kinematics<PHYS, TAB>(P, E, g, gid);
    const int level_idx0 = E.level_idx;
    const float level0 = E.level;
    reset_params<DR, TAB>(P, E, g);
    // reset_observe does not read the level; keep the redrawn one
    (void)level_idx0; (void)level0;
    reset_observe<NOISE, 0>(P, E, g, stale, out);
}

// ------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------
template <bool NOISE>
__device__ __forceinline__ void write_obs(float* __restrict__ dst, uint32_t i, const float* o) {
    constexpr int OD = NOISE ? 34 : 42;
    float2* d2 = reinterpret_cast<float2*>(dst + (size_t)i * OD);
#pragma unroll
    for (int k = 0; k < OD / 2; ++k) d2[k] = make_float2(o[2 * k], o[2 * k + 1]);
}

// Compile-time view of the env-step shape.  SPEC 1 is the reference default for the Bullet envs
// (aggregate_phy_steps 2, obs_rate 2, buf_size 2, latency + motor dynamics on): the shape fields
// of a local KParams copy become constants, so the sub-step loop unrolls, the sensor-call parity
// and the latency-ring index resolve statically and the dead sub-step draws drop out.
template <int SPEC>
__device__ __forceinline__ KParams shape_view(const KParams& P) {
    KParams Q = P;
    if (SPEC == 1 || SPEC == 2) {
        Q.agg = 2; Q.obs_rate = 2; Q.buf_size = 2; Q.use_latency = 1; Q.use_motor_dyn = 1; Q.held_persistent = 0;
    }
    if (SPEC == 1) { Q.num_drones = 1; Q.downwash_on = 0; }   // single drones: formation code drops out
    return Q;
}

// ---- phase timeline instrumentation (tools/timeline.py; -DCF2_TIMING builds only) ----
#ifdef CF2_TIMING
__device__ uint64_t* g_cf2_timing;   // [waves][16]: 0 hw id, 1 realtime start, 2 realtime end, 3.. memtime stamps
__device__ __forceinline__ uint64_t* timing_row() {
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    return g_cf2_timing ? g_cf2_timing + (size_t)wave * 16 : nullptr;
}
#define TSTAMP(k)                                                                              \
    do {                                                                                       \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();                                      \
        uint64_t* r_ = timing_row();                                                           \
        const int first_ = __ffsll((unsigned long long)__builtin_amdgcn_read_exec()) - 1;      \
        if (r_ && (int)(threadIdx.x & 63) == first_) r_[3 + (k)] = t_;                         \
    } while (0)
#define TREADY(...) asm volatile("" ::__VA_ARGS__)
#else
#define TSTAMP(k) do { } while (0)
#define TREADY(...) do { } while (0)
#endif

// P with the sensor model's parameters re-read from the kernarg segment (the final sensor call of
// the large-N step kernel: the values are the same, their registers are free during the physics)
__device__ __forceinline__ KParams late_sensor(const KParams& P) {
    KParams Q = P;
    const KernargParams k = kernarg_params();
    Q.pos_std = k->pos_std; Q.pos_unif = k->pos_unif; Q.vel_std = k->vel_std; Q.rot_std = k->rot_std;
    Q.rot_unif = k->rot_unif; Q.pgd = k->pgd; Q.sbgd = k->sbgd; Q.gyro_rw = k->gyro_rw; Q.gyro_ton = k->gyro_ton;
    Q.lpf_gain = k->lpf_gain; Q.lpf_ratio = k->lpf_ratio;
    return Q;
}

// the late_* copies when L, else the argument itself (no copy of the 624-byte block: a
// conditional expression would materialise one, and that changed the small-N kernel's code)
template <bool L> __device__ __forceinline__ decltype(auto) late_epilogue_if(const KParams& P) {
    if constexpr (L) return late_epilogue(P); else return (P);
}
template <bool L> __device__ __forceinline__ decltype(auto) late_sensor_if(const KParams& P) {
    if constexpr (L) return late_sensor(P); else return (P);
}
template <bool L> __device__ __forceinline__ decltype(auto) late_physics_if(const KParams& P) {
    if constexpr (L) return late_physics(P); else return (P);
}
template <bool L> __device__ __forceinline__ decltype(auto) late_outputs_if(const StepIO& io) {
    if constexpr (L) return late_outputs(io); else return (io);
}
// One env-step of env i (aggregate_phy_steps physics sub-steps, observation, reward, done);
// returns whether the env finished and must be auto-reset.
// What an auto-reset consumes from the finished episode (handed to the resetting lane in LDS, so
// the reset issues no global load behind the step's store burst)
struct ResetSeed {
    float wb[3], bias[3], ou[4], level;
    int level_idx;
    uint32_t ctr;
};
enum { SEED_WORDS = 13 };

// The env-step on a loaded Env.  STORE: write the state back (the one-step kernel: the physics
// state as soon as it is final, the rest at the end); the fused rollout keeps it in registers.
// HD (small-N kernel, reference-default shape with sensor noise): the draws after the first
// sub-step come from the helper waves' LDS table (hd = its column of this env, HD_* layout); the
// env wave joins the helpers' LDS barrier before its second sub-step.
template <bool NOISE, bool DR, int PHYS, bool STORE, bool SKIP_RESETTING = false, bool HD = false, int ST_AUX = 0,
          bool LATEP = false, bool LATEX = false>
// LATEP: the epilogue's, the final sensor call's parameters and the output pointers re-read where
// used (step_kernel, collect_kernel); LATEX: the epilogue's, the sensor call's and the physics
// sub-steps' parameters (the fused rollout, whose output pointers change per env-step)
__device__ __forceinline__ bool step_env_body(const KParams& P, const StepIO& io, uint32_t i, Env& E,
                                              float* __restrict__ obs_row, ResetSeed& rs, const double* hj_grid,
                                              const float* hd = nullptr) {
    constexpr int OL = NOISE ? 13 : 17;
    constexpr int OD = 2 * (OL + 4);
    const uint32_t gid = P.gid_off + i;
    const float4 a4 = reinterpret_cast<const float4*>(io.act)[i];
    TREADY("v"(E.p[0]), "v"(E.obs_prev[OL - 1]), "v"(E.hact[1][3]), "v"(E.K[3]), "v"(a4.w), "v"(E.rng));
    TSTAMP(1);   // every state load has landed
    const float a[4] = {a4.x, a4.y, a4.z, a4.w};
    const Keys K = make_keys(P.key0, P.key1);
    const Rng g{K, E.rng, gid, TAG_STEP};
    // reference-default shape: the final (full) sensor call's blocks are drawn up front (RowRng)
    const bool pre_final = !HD && NOISE && P.agg == 2 && P.obs_rate == 2;
    const uint32_t* hdw = reinterpret_cast<const uint32_t*>(hd);
    const uint32_t fbase = 8u + 8u * (uint32_t)P.agg;
    if (pre_final) {
        uint32_t* row = reinterpret_cast<uint32_t*>(obs_row);
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const U4 u = g.block(fbase + b);
            float z0, z1, z2, z3;
            box_muller(u.x, u.y, z0, z1);
            box_muller(u.z, u.w, z2, z3);
            row[4 * b] = __float_as_uint(z0); row[4 * b + 1] = __float_as_uint(z1);
            row[4 * b + 2] = __float_as_uint(z2); row[4 * b + 3] = __float_as_uint(z3);
        }
        {
            const U4 u = g.block(fbase + 4);
            float z0, z1;
            box_muller(u.x, u.y, z0, z1);
            row[16] = __float_as_uint(z0); row[17] = __float_as_uint(z1); row[18] = u.z; row[19] = u.w;
        }
        {
            const U4 u = g.block(fbase + 5);
            row[20] = u.x; row[21] = u.y; row[22] = u.z; row[23] = u.w;
        }
    }
    if (PHYS == PHYS_BULLET_T) {
        euler_from_quat(E.q, E.rpy);
        const M3 R = rotmat(E.q);
        mtv(R, E.w, E.wb);
    } else {
#pragma unroll
        for (int k = 0; k < 3; ++k) E.wb[k] = E.w[k];
    }
    const float level_used = E.level;
    // disturbance (once per env-step, held for all sub-steps)
    float d[3] = {0.0f, 0.0f, 0.0f};
    switch (P.dstb_mode) {
    case DSTB_EXTERNAL_T:
#pragma unroll
        for (int k = 0; k < 3; ++k) d[k] = io.dstb[(size_t)i * 3 + k];
        break;
    case DSTB_UNIFORM_T: {
        const U4 u = g.block(0);
        const uint32_t uu[3] = {u.x, u.y, u.z};
#pragma unroll
        for (int k = 0; k < 3; ++k)
            d[k] = (float)(-P.uni_hi[k] + (P.uni_hi[k] - -P.uni_hi[k]) * (double)u01(uu[k]));
        break;
    }
    case DSTB_CONST_T:
#pragma unroll
        for (int k = 0; k < 3; ++k) d[k] = E.dstb[k];
        break;
    case DSTB_GUST_T: {
        const U4 u = g.block(0);
        if (E.gust_left == 0 && u01(u.x) < P.gust_p) {
            E.gust_left = P.gust_dur;
            const float mag = P.gust_max * u01(u.y);
#pragma unroll
            for (int k = 0; k < 3; ++k) E.dstb[k] = ((u.z >> k) & 1u ? -1.0f : 1.0f) * mag * P.umax[k];
        }
        if (E.gust_left > 0) {
#pragma unroll
            for (int k = 0; k < 3; ++k) d[k] = E.dstb[k];
            E.gust_left -= 1;
        } else {
#pragma unroll
            for (int k = 0; k < 3; ++k) E.dstb[k] = 0.0f;
        }
        break;
    }
    case DSTB_HJ_T: {
        const int t = P.level_mode == LEVEL_FIXED_T ? P.tab->table_of_level[0] : P.tab->table_of_level[E.level_idx & 31];
        if (t >= 0 && P.V != nullptr) {
            float e[3];
            quat2euler(E.q, e);
            const double st[6] = {(double)e[0], (double)e[1], (double)e[2], (double)E.wb[0], (double)E.wb[1], (double)E.wb[2]};
            // the node's sign bits were derived from its 7 taps once per table (cf2_bind_hj_tables):
            // one byte gathered per env-step instead of 7 scattered floats of the 45.6 MB table
            int idx[6];
            const int c = hj_node(st, hj_grid, idx);
            const unsigned bits = P.hj_bits[(size_t)t * HJ_TABLE + (size_t)c];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const float dm = (float)((double)E.level * (double)P.umax_d[k]);
                d[k] = (bits >> k) & 1u ? -dm : dm;
            }
        }
        break;
    }
    default: break;
    }
#pragma unroll 4
    for (int s = 0; s < P.agg; ++s) {
        float on[4];
        if (HD && s == 1) normals<4>(RowRng<64>{hdw + HD_OU1 * 64, 2}, 2, on);
        else normals<4>(g, 1 + s, on);
        float dw = 0.0f;
        if (PHYS == PHYS_BULLET_T && P.num_drones > 1 && P.downwash_on)
            dw = downwash(P, E.p, gid % (uint32_t)P.num_drones);   // mates' positions before this sub-step
        if (PHYS == PHYS_BULLET_T) bullet_substep(late_physics_if<LATEX>(P), E, a, d, on, E.ep_step == 0 && s == 0 && !E.props_on, dw);
        else simple_substep(late_physics_if<LATEX>(P), E, a, on);
        float dummy[17];
        // a sub-step's held measurement reaches an observation only if the final measurement
        // of the env-step is not a full one (aggregate_phy_steps % obs_rate != 0)
        if (HD && s == 0) {
            // compute_observation of this full call with its held part dead: the gyro update alone
            lds_barrier();                                   // the helper waves' draws are in LDS
            float ng[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) ng[k] = hd[(HD_GYRO0 + k) * 64];
            gyro_update(P, E, ng);
        } else if (HD && s == 1) {
            compute_observation<NOISE>(P, E, RowRng<64>{hdw + HD_GYRO1 * 64, 16}, 16, E.ep_step * P.agg + s, dummy, false);
        } else {
            compute_observation<NOISE>(P, E, g, 8 + 8 * s, E.ep_step * P.agg + s, dummy, P.held_persistent != 0);
        }
    }
    // the history (o_{k-1}, last actions) is only read by compute_history: the one-step kernel
    // loads it after the physics, so its 21 registers are not live across the sub-steps (the final
    // sensor call hides the load latency; -0.6 us at 262144 envs)
    if (STORE) load_hist<NOISE>(Tile(io.sf, P.N, i), E);
    float onx[17];
    TREADY("v"(E.q[3]), "v"(E.lpf[2]));
    TSTAMP(2);   // physics sub-steps done
    if (HD) {
        compute_observation<NOISE>(P, E, RowRng<64>{hdw + HD_FINAL * 64, fbase}, fbase, (E.ep_step + 1) * P.agg, onx);
    } else if (pre_final) {
        const RowRng<1> gr{reinterpret_cast<const uint32_t*>(obs_row), fbase};
        compute_observation<NOISE>(late_sensor_if<LATEP || LATEX>(P), E, gr, fbase, (E.ep_step + 1) * P.agg, onx);
    } else {
        compute_observation<NOISE>(late_sensor_if<LATEP || LATEX>(P), E, g, fbase, (E.ep_step + 1) * P.agg, onx);
    }
    // LATEP (the large-N step kernel): the epilogue's parameters re-read here (late_epilogue)
    const auto& PL = late_epilogue_if<LATEP || LATEX>(P);
    const bool term = compute_done(PL, E);
    E.ep_step += 1;
    const bool trunc = P.max_steps > 0 && E.ep_step >= P.max_steps && !term;
    const bool done = term || trunc;
    const bool do_reset = done && P.auto_reset;
    // the physics state is final now: store it early so its registers free up before the
    // epilogue.  SKIP_RESETTING (the small-N kernel, whose reset stores follow an LDS-only
    // barrier): an env that auto-resets is not stored, its reset writes every group stored here,
    // so no two waves store one group in one launch.  The large-N kernel stores it anyway: its
    // resets follow __syncthreads, whose workgroup-scope release/acquire orders these stores before
    // the reset waves' stores to the same groups (skipping them cost 0.6 us there)
    if (STORE && !(SKIP_RESETTING && do_reset)) store_core<NOISE, DR, PHYS, ST_AUX>(P, io.sf, i, E);
    const auto& IL = late_outputs_if<LATEP>(io);
    {
        const float r = compute_reward(PL, E, a, term);
        const float cost = IL.cost ? compute_cost(PL, E) : 0.0f;    // info['cost'] only when asked for
        IL.rew[i] = r;
        IL.done[i] = (uint8_t)done;
        if (IL.trunc) IL.trunc[i] = (uint8_t)trunc;
        if (IL.cost) IL.cost[i] = cost;
        if (IL.level) IL.level[i] = level_used;
    }
    {
        float o[OD];
        compute_history<NOISE>(P, E, onx, o);
        // the block's obs rows are staged in LDS and written out coalesced by the kernel; a
        // reset env's row is overwritten there by its reset observation
#pragma unroll
        for (int k = 0; k < OD; k += 2)
            *reinterpret_cast<float2*>(obs_row + k) = make_float2(o[k], o[k + 1]);
        if (do_reset && IL.final_obs) write_obs<NOISE>(IL.final_obs, i, o);
    }
    if (do_reset) {
#pragma unroll
        for (int k = 0; k < 3; ++k) { rs.wb[k] = E.wb[k]; rs.bias[k] = NOISE ? E.bias[k] : 0.0f; }
#pragma unroll
        for (int k = 0; k < 4; ++k) rs.ou[k] = E.ou[k];
        rs.level = E.level;
        rs.level_idx = E.level_idx;
        rs.ctr = E.rng;
    }
    E.rng += 1;
    if (STORE && !(SKIP_RESETTING && do_reset)) store_tail<NOISE, ST_AUX>(P, io.sf, i, E);
    TSTAMP(3);   // epilogue issued
    return do_reset;
}

template <bool NOISE, bool DR, int PHYS, bool SKIP_RESETTING = false, bool HD = false, int ST_AUX = 0,
          bool LATEP = false>
__device__ __forceinline__ bool step_env(const KParams& P, const StepIO& io, uint32_t i, float* __restrict__ obs_row,
                                         ResetSeed& rs, const double* hj_grid, const float* hd = nullptr) {
    Env E;
    // every state load is issued before the first state store: on gfx9 vmcnt also counts stores,
    // so a load issued after the state stores would wait for the whole store burst to drain (the
    // history is loaded after the physics sub-steps, still ahead of store_core, in step_env_body)
    load_env<NOISE, DR, PHYS>(P, io.sf, i, E, P.need_level || io.level != nullptr, /*with_hist=*/false);
    return step_env_body<NOISE, DR, PHYS, true, SKIP_RESETTING, HD, ST_AUX, LATEP>(P, io, i, E, obs_row, rs, hj_grid, hd);
}

// Reset one env in place: reads only what a reset consumes from the finished episode (the
// stale body rates for the gyro LPF, the never-reset gyro bias and OU state, the RNG counter
// and the disturbance level), writes the reset observation row and the whole state.
template <bool NOISE, bool DR, int PHYS>
__device__ __forceinline__ void reset_one(const KParams& P, float* __restrict__ sf, uint32_t i, float* __restrict__ obs) {
    constexpr int OD = NOISE ? 34 : 42;
    const Tile T(sf, P.N, i);
    Env E;
    const F4 g0 = T.ld(0), g1 = T.ld(1), g2 = T.ld(2), g3 = T.ld(3), go = T.ld(G_OU);
    const float q[4] = {g0.w, g1.x, g1.y, g1.z}, w[3] = {g2.z, g2.w, g3.x};
    if (PHYS == PHYS_BULLET_T) {
        const M3 R = rotmat(q);
        mtv(R, w, E.wb);
    } else {
#pragma unroll
        for (int k = 0; k < 3; ++k) E.wb[k] = w[k];
    }
    if (NOISE) {
        const F4 b = T.ld(G_BIAS);
        E.bias[0] = b.x; E.bias[1] = b.y; E.bias[2] = b.z;
    }
    E.ou[0] = go.x; E.ou[1] = go.y; E.ou[2] = go.z; E.ou[3] = go.w;
    const uint32_t rng_ctr = (uint32_t)bi(g3.z);
    E.rng = rng_ctr;
    E.level = T.ld(G_LEVEL).w;
    E.level_idx = bi(T.ld(G_LEVEL_IDX).x);
    float o[OD];
    const Keys K = make_keys(P.key0, P.key1);
    const Rng g{K, rng_ctr, P.gid_off + i, TAG_RESET};
    reset_env<NOISE, DR, PHYS>(P, E, g, P.gid_off + i, o);
    E.rng = rng_ctr + 1;
    if (obs) write_obs<NOISE>(obs, i, o);
    store_env<NOISE, DR, PHYS>(P, sf, i, E, true);
}

// The state groups an auto-reset writes, in three sets (their union is store_env(params_dirty)):
//   kinematics: pose, velocities, counters (rng = ctr + 1), motor state, OU state (inherited from
//               the finished episode), latency ring, rpy (Simple)       -> groups 0-6(+ring), 12, 28
//   history:    gyro bias (+ gust_left 0), held measurement, action history, o_{k-1} + gyro LPF
//                                                                        -> groups 10, 14-19, 21-23
//   params:     domain randomisation, disturbance, level                -> groups 13, 24-27, 29
template <int PHYS>
__device__ __forceinline__ void store_reset_kinematics(const KParams& P, const Tile& T, const Env& E, const float ou[4],
                                                       uint32_t ctr) {
    T.st(0, f4(E.p[0], E.p[1], E.p[2], E.q[0]));
    T.st(1, f4(E.q[1], E.q[2], E.q[3], E.v[0]));
    T.st(2, f4(E.v[1], E.v[2], E.w[0], E.w[1]));
    const int fl = (E.aidx & 15) | (1 << 4) | (1 << 5) | (E.la_view << 6) | (E.props_on << 7);   // halias0/1 = 1
    T.st(G_CORE3, f4(E.w[2], ib(0), ib((int)(ctr + 1u)), ib(fl)));
    T.st(G_MOTOR, f4(E.x[0], E.x[1], E.x[2], E.x[3]));
    if (P.use_motor_dyn) T.st(G_MOTOR_LO, f4(0.0f, 0.0f, 0.0f, 0.0f));
    T.st(G_OU, f4(ou[0], ou[1], ou[2], ou[3]));
#pragma unroll
    for (int r = 0; r < 4; ++r)
        if (r < P.buf_size) T.st(G_ABUF + r, f4(E.abuf[r][0], E.abuf[r][1], E.abuf[r][2], E.abuf[r][3]));
    if (PHYS == PHYS_SIMPLE_T) T.st(G_RPY, f4(E.rpy[0], E.rpy[1], E.rpy[2], 0.0f));
}
template <bool NOISE>
__device__ __forceinline__ void store_reset_history(const KParams& P, const Tile& T, const Env& E) {
    if (NOISE || gust_mode(P))
        T.st(G_BIAS, f4(NOISE ? E.bias[0] : 0.0f, NOISE ? E.bias[1] : 0.0f, NOISE ? E.bias[2] : 0.0f, ib(0)));
    if (NOISE && P.held_persistent) {
        T.st(G_HELD, f4(E.held[0], E.held[1], E.held[2], E.held[3]));
        T.st(G_HELD + 1, f4(E.held[4], E.held[5], E.held[6], E.held[7]));
        T.st(G_HELD + 2, f4(E.held[8], E.held[9], 0.0f, 0.0f));
    }
    T.st(G_HACT, f4(E.hact[0][0], E.hact[0][1], E.hact[0][2], E.hact[0][3]));
    T.st(G_HACT + 1, f4(E.hact[1][0], E.hact[1][1], E.hact[1][2], E.hact[1][3]));
    store_obs_prev<NOISE>(T, E);
}
template <bool DR>
__device__ __forceinline__ void store_reset_params(const KParams& P, const Tile& T, const Env& E) {
    if (dstb_stored(P)) T.st(G_DSTB, f4(E.dstb[0], E.dstb[1], E.dstb[2], 0.0f));
    if (DR) {
        T.st(G_PARAM, f4(E.dt, E.m, E.J[0], E.J[1]));
        T.st(G_PARAM + 1, f4(E.J[2], E.k0, E.k1, E.B[0]));
        T.st(G_PARAM + 2, f4(E.B[1], E.B[2], E.B[3], E.K[0]));
    }
    T.st(G_LEVEL, f4(E.K[1], E.K[2], E.K[3], E.level));
    T.st(G_LEVEL_IDX, f4(ib(E.level_idx), 0.0f, 0.0f, 0.0f));
}

// One quarter of an auto-reset (block_epilogue runs the four roles on four waves at once; the
// union of their stores is store_env(params_dirty) and of their row writes the reset
// observation, as reset_env + store_env produce them):
//   0: kinematics, motor state, ring           -> store_reset_kinematics
//   1: kinematics + the first sensor call      -> obs row o_0 | A_0
//   2: kinematics + the second sensor call     -> obs row o_1 | A_1; store_reset_history
//   3: domain randomisation, disturbance, level -> store_reset_params
// Roles 1 and 2 recompute the reset pose from the same table entries, so the critical path is one
// pose + one sensor call instead of the whole reset.
template <bool NOISE, bool DR, int PHYS, int TAB = 0>
__device__ __forceinline__ void reset_role(const KParams& P, float* __restrict__ sf, uint32_t i, const ResetSeed& rs,
                                           const TableRng& g, float* __restrict__ obs_row, uint32_t role) {
    constexpr int OL = NOISE ? 13 : 17;
    const Tile T(sf, P.N, i);
    const uint32_t gid = P.gid_off + i;
    Env E;
    TSTAMP(6);   // role start (after the table-draw barrier)
#pragma unroll
    for (int k = 0; k < 3; ++k) { E.wb[k] = rs.wb[k]; E.bias[k] = rs.bias[k]; }
    const float stale[3] = {rs.wb[0], rs.wb[1], rs.wb[2]};
    if (role == 3) {
        E.level = rs.level;
        E.level_idx = rs.level_idx;
        reset_params<DR, TAB>(P, E, g);
        store_reset_params<DR>(P, T, E);
        return;
    }
    reset_kinematics<PHYS, TAB>(P, E, g, gid);
    TREADY("v"(E.q[3]), "v"(E.w[0]));
    TSTAMP(7);   // reset pose computed
    if (role == 0) {
        store_reset_kinematics<PHYS>(P, T, E, rs.ou, rs.ctr);
        return;
    }
    if (role == 1) {
        float o[OL + 4];
        reset_observe<NOISE, 1>(P, E, g, stale, o);
#pragma unroll
        for (int k = 0; k < OL + 4; ++k) obs_row[k] = o[k];
        return;
    }
    float o[2 * (OL + 4)];
    reset_observe<NOISE, 2>(P, E, g, stale, o);
#pragma unroll
    for (int k = OL + 4; k < 2 * (OL + 4); ++k) obs_row[k] = o[k];
    TREADY("v"(o[2 * (OL + 4) - 1]));
    TSTAMP(8);   // role 2: second sensor call + history done
    store_reset_history<NOISE>(P, T, E);
}

// End of a block's env-step: list the finished envs (wave ballots into per-wave lists), reset
// them block-cooperatively (see step_kernel) and write the block's obs rows out coalesced.  Every
// thread of the block calls it.
template <bool NOISE, bool DR, int PHYS, uint32_t B, uint32_t C, int TAB = 0>
__device__ __forceinline__ void block_epilogue(const KParams& P, const StepIO& io, uint32_t base, uint32_t tid,
                                               bool do_reset, const ResetSeed& rs, float* s_obs, uint32_t* s_list,
                                               uint32_t* s_rand, uint32_t* s_wcnt) {
    constexpr int OD = NOISE ? 34 : 42;
    constexpr uint32_t W = B / 64u;
    if (P.auto_reset) {
        // finished envs listed per wave (ballot; no atomics, no counter to initialise): wave w's
        // resets at s_list[64 w ..], its count in s_wcnt[w]; global reset order is wave-major
        const uint64_t m = __ballot(do_reset);
        const uint32_t wv = tid >> 6, lane = tid & 63u;
        if (lane == 0) s_wcnt[wv] = (uint32_t)__popcll(m);
        if (do_reset) {
            s_list[64u * wv + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = tid;
            // the seed is parked in the env's own LDS obs row (its final obs is already in
            // final_obs; the row is overwritten by the reset observation after the seed is read)
            uint32_t* row = reinterpret_cast<uint32_t*>(s_obs + tid * OD);
#pragma unroll
            for (int k = 0; k < 3; ++k) { row[k] = __float_as_uint(rs.wb[k]); row[3 + k] = __float_as_uint(rs.bias[k]); }
#pragma unroll
            for (int k = 0; k < 4; ++k) row[6 + k] = __float_as_uint(rs.ou[k]);
            row[10] = __float_as_uint(rs.level);
            row[11] = (uint32_t)rs.level_idx;
            row[12] = rs.ctr;
        }
        __syncthreads();
        TSTAMP(4);   // block barrier passed
        uint32_t wc[W], cnt = 0;
#pragma unroll
        for (uint32_t w = 0; w < W; ++w) { wc[w] = s_wcnt[w]; cnt += wc[w]; }
        // global reset position -> block-local env index
        auto env_at = [&](uint32_t p) -> uint32_t {
            uint32_t w = 0;
#pragma unroll
            for (uint32_t k = 0; k + 1 < W; ++k)
                if (w == k && p >= wc[k]) { p -= wc[k]; w = k + 1; }
            return s_list[64u * w + p];
        };
        // Resets run in chunks of C envs.  Their ~26 Philox blocks per env are drawn by every
        // thread of the block in parallel into LDS; then the reset math runs on the table, split
        // by role over the four waves.  (On one lane each, the draws made the reset tail, which
        // every wave of the block waits for, about as long as the env-step itself; one wave running
        // whole resets instead of the role split: 41.2 vs 40.1 us at 262 144 envs.)
        static_assert(B == 256u, "four waves, one reset role each");
        for (uint32_t c0 = 0; c0 < cnt; c0 += C) {
            const uint32_t nc = cnt - c0 < C ? cnt - c0 : C;
            // role lanes take their seed now: this chunk's rows are only overwritten after the
            // barrier below (and other chunks' roles never touch them), so no extra barrier
            const uint32_t rl = tid & 63u, role = ((tid >> 6) + blockIdx.x) & 3u;
            const bool act = rl < nc;
            ResetSeed q;
            uint32_t t = 0;
            if (act) {
                t = env_at(c0 + rl);
                const uint32_t* row = reinterpret_cast<const uint32_t*>(s_obs + t * OD);
#pragma unroll
                for (int c = 0; c < 3; ++c) { q.wb[c] = __uint_as_float(row[c]); q.bias[c] = __uint_as_float(row[3 + c]); }
#pragma unroll
                for (int c = 0; c < 4; ++c) q.ou[c] = __uint_as_float(row[6 + c]);
                q.level = __uint_as_float(row[10]);
                q.level_idx = (int)row[11];
                q.ctr = row[12];
            }
            {
                const Keys K = make_keys(P.key0, P.key1);
                for (uint32_t w = tid; w < nc * RESET_SLOTS; w += B) {
                    const uint32_t sl = w / nc, e = w - sl * nc;
                    const uint32_t te = env_at(c0 + e);
                    const uint32_t ctr = reinterpret_cast<const uint32_t*>(s_obs + te * OD)[12];
                    U4 u = philox(K, reset_block_of_slot((int)sl), ctr, P.gid_off + base + te, TAG_RESET);
                    if (reset_slot_normal_xy((int)sl)) {
                        float z0, z1;
                        box_muller(u.x, u.y, z0, z1);
                        u.x = __float_as_uint(z0); u.y = __float_as_uint(z1);
                    }
                    if (reset_slot_normal_zw((int)sl)) {
                        float z2, z3;
                        box_muller(u.z, u.w, z2, z3);
                        u.z = __float_as_uint(z2); u.w = __float_as_uint(z3);
                    }
                    uint32_t* qq = s_rand + sl * 4 * C + e;
                    qq[0] = u.x; qq[C] = u.y; qq[2 * C] = u.z; qq[3 * C] = u.w;
                }
            }
            __syncthreads();
            // the four waves split each reset by role (reset_role); the role of a wave rotates
            // with the block index so the co-resident blocks' roles spread over the SIMDs
            if (act) {
                const TableRng tg{s_rand + rl, C};
                reset_role<NOISE, DR, PHYS, TAB>(P, io.sf, base + t, q, tg, s_obs + t * OD, role);
            }
            __syncthreads();     // the next chunk reuses s_rand
        }
        TSTAMP(12);  // every reset chunk done
    } else {
        __syncthreads();         // every obs row of the block is in LDS
    }
    write_obs_rows<B, OD, B>(io.obs + (size_t)base * OD, s_obs, P.N - base < B ? P.N - base : B, tid);
}

// The delta exchange's pack fused into the large-N env-step (cf2_step_packed above 32 768 envs):
// after block_epilogue the block's 256 rows are final in s_obs (reset rows hold the reset
// observation), so every thread writes its share of the block's o_k run, and each wave (one 64-env
// pack block) its two bitmap words, its block-table word and its resets' side entries.
template <uint32_t OL, uint32_t OD, uint32_t B>
__device__ __forceinline__ void pack_epilogue_block(const PackIO& X, uint32_t n, uint32_t base, uint32_t tid,
                                                    bool do_reset, const float* s_obs) {
    typedef float f4x __attribute__((ext_vector_type(4)));
    const PackLayout L{n, OL, X.cap};
    uint32_t* pk = X.pk;
    const uint32_t lane = tid & 63u, wbase = base + (tid & ~63u);
    const uint64_t m = __ballot(do_reset);
    uint32_t first = 0u;
    if (lane == 0 && m) first = pack_alloc(L, X.scratch, (uint32_t)__popcll(m));
    const uint32_t nvalid = n - base < B ? n - base : B;
    float* dst = reinterpret_cast<float*>(pk + L.o_slab()) + (size_t)base * OL;
    if (nvalid == B && ((uintptr_t)dst & 15u) == 0) {
        f4x* d4 = reinterpret_cast<f4x*>(dst);
        for (uint32_t c = tid; c < B * OL / 4u; c += B) {
            f4x v;
#pragma unroll
            for (uint32_t e = 0; e < 4u; ++e) {
                const uint32_t f = 4u * c + e, r = f / OL;
                v[e] = s_obs[r * OD + OL + 4u + (f - r * OL)];
            }
            d4[c] = v;
        }
    } else {
        for (uint32_t f = tid; f < nvalid * OL; f += B) {
            const uint32_t r = f / OL;
            dst[f] = s_obs[r * OD + OL + 4u + (f - r * OL)];
        }
    }
    if (wbase < n) {
        uint32_t* bits = pk + L.bits();
        if (lane == 0) bits[wbase / 32u] = (uint32_t)m;
        if (lane == 1 && wbase + 32u < n) bits[wbase / 32u + 1u] = (uint32_t)(m >> 32);
        first = __shfl(first, 0);
        if (lane == 0) pk[L.btab() + wbase / XB_PACK] = first;
        const uint32_t slot =
            pack_entry_slot(L, wbase / XB_PACK, (uint32_t)__popcll(m & ((1ull << lane) - 1ull)), first);
        if (do_reset && slot != PACK_DROPPED) {
            uint32_t* e = pk + L.side() + slot * L.entry();
            e[0] = base + tid;
            const float* row = s_obs + tid * OD;
            float* ef = reinterpret_cast<float*>(e + 1);
#pragma unroll
            for (uint32_t k = 0; k < OL + 4u; ++k) ef[k] = row[k];     // o_0 and A (= A_0)
        }
    }
}

// Launch shape of the large-N env kernels: 256-thread blocks of 256 envs (= the auto-reset
// compaction group), 3 waves per SIMD (<= 168 VGPRs, <= 53 KB LDS per block); resets drawn and run
// in chunks of 32
constexpr uint32_t STEP_BLOCK = 256, STEP_MIN_WAVES = 3, RESET_CHUNK = 32;
// Step kernel: one lane per env.  Auto-reset is compacted per block: with random actions a few
// % of envs finish per step, so nearly every wave would hold one and run the whole reset path
// divergently.  Finished envs are listed in LDS and reset by the fewest waves after a block
// barrier; their state rows were just written by this block and are still in L2, so the reset's
// scattered SoA accesses cost no extra HBM traffic (a separate reset kernel pays ~60 B per
// 4-byte field access for them).
template <bool NOISE, bool DR, int PHYS, int SPEC, int ST_AUX = 0>
__global__ void __launch_bounds__(STEP_BLOCK, STEP_MIN_WAVES) step_kernel(KParams P0, StepIO io, PackIO X) {
    const KParams P = shape_view<SPEC>(P0);
    // Issue priority: the blocks that start only after the first residency round (the partial
    // last round at 262 144 envs) run mostly alone on their SIMDs and end the kernel; their waves
    // get the issue slots first, so they overlap the tail of the first round (-1 us measured;
    // starting the first round's co-resident blocks 2k-8k cycles apart instead: equal or slower).
    if (blockIdx.x >= P0.late_block) __builtin_amdgcn_s_setprio(3);
    else __builtin_amdgcn_s_setprio(1);
#ifdef CF2_TIMING
    if (uint64_t* r = timing_row()) {
        if ((threadIdx.x & 63) == 0) {
            const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_ID
            const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);   // XCC_ID
            r[0] = ((uint64_t)xcc << 32) | hw;
            r[1] = __builtin_amdgcn_s_memrealtime();
            r[3] = __builtin_amdgcn_s_memtime();
        }
    }
#endif
    constexpr int OD = NOISE ? 34 : 42;
    constexpr uint32_t B = STEP_BLOCK, C = RESET_CHUNK;
    __shared__ __align__(16) float s_obs[B * OD];          // the block's obs rows, global layout
    __shared__ uint32_t s_list[B];                         // queue: block-local env index
    __shared__ uint32_t s_rand[RESET_SLOTS * 4 * C];       // the chunk's Philox blocks, [slot][word][env]
    __shared__ uint32_t s_wcnt[B / 64];                    // finished envs per wave
    const uint32_t tid = threadIdx.x, base = blockIdx.x * B, i = base + tid;
    bool do_reset = false;
    ResetSeed rs;
    __shared__ double s_hjgrid[6 * HJ_PTS];
    if (P.dstb_mode == DSTB_HJ_T) stage_hj_grid(P.tab->hj_grid, s_hjgrid);     // uniform branch
    if (i < P.N) do_reset = step_env<NOISE, DR, PHYS, false, false, ST_AUX, true>(P, io, i, s_obs + tid * OD, rs, s_hjgrid);
    block_epilogue<NOISE, DR, PHYS, B, C, 2>(P, io, base, tid, do_reset, rs, s_obs, s_list, s_rand, s_wcnt);
    if (X.pk) pack_epilogue_block<NOISE ? 13u : 17u, (uint32_t)OD, B>(X, P.N, base, tid, do_reset, s_obs);
#ifdef CF2_TIMING
    TSTAMP(5);   // resets done
    if (uint64_t* r = timing_row())
        if ((threadIdx.x & 63) == 0) r[2] = __builtin_amdgcn_s_memrealtime();
#endif
}

// Fused collect step: step_kernel's env-step, then the actor-critic
// forward on the block's new observations, one launch per env-step of the collect loop.  It
// replaces the pair env.step (algs/iwpg/iwpg.py:380) + ac.step (:377, algs/core.py:371-395) of
// IWPGAlgorithm.roll_out as the loop runs them back to back (policy of step t+1 right after the
// env-step of step t).  With two launches the policy kernel re-reads the obs rows from memory
// and runs alone, bound by vector issue, while the env-step leaves ~70 % of the issue slots idle
// waiting on memory; here a block's policy phase runs beside the env phases
// of the blocks sharing its CU.
//   * env phase: exactly step_kernel's (same device code: the obs, rewards, flags, final obs and
//     state are bit-identical to cf2_step's);
//   * the block's 256 obs rows are still in LDS after the write-out: each wave reads its 64 rows
//     (4 row tiles) as MFMA B operands into registers, then the block's LDS is re-used for the
//     packed fragments (52.6 KB: all but layer 3's 8 KB, which the waves read from global memory,
//     L1/L2-resident), so the kernel keeps step_kernel's 3 blocks per CU (<= 53 KB each);
//   * policy phase: policy_layers / policy_emit of cf2sim_policy.h on each of the wave's 4 row
//     tiles: the same instructions as policy_kernel, so act / val / logp are bit-identical to
//     cf2_policy_forward on the same observations.
// Built for the bench workload's shape (noise on: 34-wide observations; bf16x3 products) at
// N > 32 768 (256 envs per block); other configs return hipErrorNotSupported and the caller runs
// the two launches.
// Delaying a third of the first round's blocks by 4k / 10k / 20k cycles, so that co-resident
// blocks reach their policy phases at different times, was slower at every delay (62.1 / 64.1 /
// 67.2 vs 61.1 us at 262 144 envs, profiles/r03_collect_ab.txt); two row tiles per forward call
// (two chains interleaved, 163 VGPRs) took the same time as one.
template <bool NOISE, bool DR, int PHYS, int SPEC>
__global__ void __launch_bounds__(STEP_BLOCK, STEP_MIN_WAVES) collect_kernel(KParams P0, StepIO io, PolicyIO pio) {
    static_assert(NOISE, "the fused collect kernel is built for the 34-wide observation");
    const KParams P = shape_view<SPEC>(P0);
    if (blockIdx.x >= P0.late_block) __builtin_amdgcn_s_setprio(3);
    else __builtin_amdgcn_s_setprio(1);
    constexpr int OD = 34;
    constexpr uint32_t B = STEP_BLOCK, C = RESET_CHUNK, W = B / 64u;
    static_assert(B == 256, "one 64-row wave per SIMD quarter of the block");
    using PK = Packed<OD, CF2_POLICY_BF16X3>;
    // LDS: the env phase's arrays, then the fragments but layer 3 (the tail from O_BIAS on moves
    // down to O_L3)
    constexpr uint32_t L3N = PK::O_BIAS - PK::O_L3, POL_WORDS = PK::TOTAL - L3N;
    constexpr uint32_t HJ_AT = (B * OD + B + RESET_SLOTS * 4 * C + W + 1) & ~1u;     // 8-B aligned
    constexpr uint32_t ENV_WORDS = HJ_AT + 2 * 6 * HJ_PTS;
    constexpr uint32_t LDS_WORDS = POL_WORDS > ENV_WORDS ? POL_WORDS : ENV_WORDS;
    static_assert(PK::O_L3 % 4 == 0 && PK::O_BIAS % 4 == 0 && PK::TOTAL % 4 == 0, "float4 staging");
    __shared__ __align__(16) float s_mem[LDS_WORDS];
    float* s_obs = s_mem;
    uint32_t* s_list = reinterpret_cast<uint32_t*>(s_mem + B * OD);
    uint32_t* s_rand = s_list + B;
    uint32_t* s_wcnt = s_rand + RESET_SLOTS * 4 * C;
    double* s_hjgrid = reinterpret_cast<double*>(s_mem + HJ_AT);
    const uint32_t tid = threadIdx.x, base = blockIdx.x * B, i = base + tid;
    bool do_reset = false;
    ResetSeed rs;
    if (P.dstb_mode == DSTB_HJ_T) stage_hj_grid(P.tab->hj_grid, s_hjgrid);     // uniform branch
    // kernel parameters re-read where used, as step_kernel (-0.8 us per env-step of the collect loop)
    if (i < P.N) do_reset = step_env<NOISE, DR, PHYS, false, false, 0, true>(P, io, i, s_obs + tid * OD, rs, s_hjgrid);
    block_epilogue<NOISE, DR, PHYS, B, C, 2>(P, io, base, tid, do_reset, rs, s_obs, s_list, s_rand, s_wcnt);
    // ---- policy phase.  Lane l of wave wv holds, for row tile c, row 64 wv + 16 c + (l & 15):
    // inputs 8 g .. 8 g + 7 (k-block 0) and 32 + g (the fp32 k-step; clamped, zero weight past D)
    const uint32_t l = tid & 63u, wv = tid >> 6, r16 = l & 15u;
    const int g = (int)(l >> 4);
    constexpr int CR = 1, NCH = 4 / CR;                       // row tiles per forward call, calls per wave
    ObsRegs<OD, CF2_POLICY_BF16X3, CR> X[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int rt = 0; rt < CR; ++rt) {
            const float* row = s_obs + (64u * wv + 16u * (uint32_t)(CR * c + rt) + r16) * OD;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float2 v = *reinterpret_cast<const float2*>(row + 8 * g + 2 * q);
                X[c].x8[rt][0][2 * q] = v.x;
                X[c].x8[rt][0][2 * q + 1] = v.y;
            }
            X[c].x1[rt][0] = row[__builtin_elementwise_min(32 + g, OD - 1)];
        }
    __syncthreads();         // every wave holds its rows: the LDS takes the fragments
    // fragment loads first; while they are in flight each lane draws the sampling noise of the
    // wave's row 64 wv + l (one Philox block per row, instead of one per row tile on all 64 lanes)
    constexpr uint32_t NQ4 = POL_WORDS / 4, NQ = (NQ4 + B - 1) / B;
    float4 stg[NQ];
    {
        const float4* src = reinterpret_cast<const float4*>(pio.w);
#pragma unroll
        for (uint32_t q = 0; q < NQ; ++q) {
            const uint32_t k = __builtin_elementwise_min(tid + q * B, NQ4 - 1u);
            stg[q] = src[k < PK::O_L3 / 4 ? k : k + L3N / 4];
        }
    }
    float ep[4];
    policy_noise(pio.key0, pio.key1, pio.counter, pio.row_offset + base + 64u * wv + l, ep);
    {
        float4* dst = reinterpret_cast<float4*>(s_mem);
#pragma unroll
        for (uint32_t q = 0; q < NQ; ++q)
            if (tid + q * B < NQ4) dst[tid + q * B] = stg[q];
    }
    __syncthreads();
    PolicyLane<OD, CF2_POLICY_BF16X3> CL;
    policy_lane_init<OD, CF2_POLICY_BF16X3>(s_mem + PK::O_L3, g, CL);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {          // unrolled: X[c] stays in registers
        int off = 0;
        asm volatile("" : "+v"(off));        // keep the fragment reads inside the loop (policy_kernel)
        const float* sw = s_mem + off;
        ObsRegs<OD, CF2_POLICY_BF16X3, CR> Xc = X[c];
        policy_standardize<OD, CF2_POLICY_BF16X3, CR>(sw + PK::O_L3, g, CL, Xc);
        f4v o[CR];
        policy_layers<OD, CF2_POLICY_BF16X3, 0, CR>(sw, sw + PK::O_L3, pio.w + PK::O_L3, (int)l, Xc, o);
#pragma unroll
        for (int rt = 0; rt < CR; ++rt) {
            const uint32_t wr = 16u * (uint32_t)(CR * c + rt) + r16, row = base + 64u * wv + wr;
            float e[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)      // row wr's noise from lane wr
                e[k] = __int_as_float(__builtin_amdgcn_ds_bpermute((int)(wr << 2), __float_as_int(ep[k])));
            if (row < P.N)
                policy_emit_eps<OD, CF2_POLICY_BF16X3, 0>(o[rt], row, g, CL, e, 1, pio.act, pio.val, pio.logp,
                                                          nullptr);
        }
    }
}

// Small N (<= 32 768 envs): the launch is as long as one wave's env-step chain, and the auto-reset
// tail used to be ~40 % of it (section 3 describes this kernel).  Each 256-thread block holds 64 envs.  Wave 0
// steps them (issue priority 3).  Waves 1-3 meanwhile compute, speculatively for all 64 envs and at
// priority 0, every part of a potential auto-reset that does not depend on the finished episode:
// a reset's draws are keyed by the env's RNG counter, which is known when the state loads, so
// they are the same Philox blocks the reset would draw after the step.
//   wave 1 (A): reset pose, velocities, motor state, latency ring    (reset_kinematics), domain
//               randomisation, disturbance, level (reset_params)
//   wave 2 (B): the pose again, the first reset sensor call's held measurement and gyro normals;
//               stages the reset observation row but for its two gyro-LPF triples
//   wave 3 (C): the pose again and the second sensor call's held part (into the staged row) and
//               gyro normals (handed to B in LDS)
// After one LDS barrier only the finished envs' work remains, on their lanes of waves 1-3: the two
// gyro updates, which need the finished episode's body rates (the gyro LPF seed) and gyro bias,
// the reset observation row, and the reset's state stores (store_reset_*).  The env wave does not
// store the state of envs that reset (step_env_body), so no group is stored twice.
// Measured and not kept: reward, cost and the per-env outputs finished by helper wave 3 from an
// LDS table after the barrier (32 768 envs 10.3 -> 11.0 us: the reset tail grew more than the env
// wave's epilogue shrank); the DR draws before the draw barrier (10.6 -> 11.2 us).
enum { SEED_SMALL = 10 };   // per finished env, wave 0 -> waves 1-3: final body rates, gyro bias, OU state
enum { C2_WORDS = 9 };      // per env, wave 3 -> wave 2: the second reset sensor call's gyro normals

// The delta exchange's pack fused into the small-N env-step (cf2_step_packed; the layout and the
// side-slot allocation are cf2sim_pack.h's, the standalone form is obs_pack_kernel): wave 2, once the
// reset rows are final (s_rrow; the other rows are final in s_obs at the block barrier), writes the
// block's bitmap words and block-table word, each lane its row's o_k (13 or 17 dword stores, the
// wave's together a contiguous run) and, for a reset row, its side entry.  The packed buffer is then
// ready for the all-gather when the env-step kernel ends: no pack kernel, no re-read of the
// observation rows.  A block with more resets than its quota asks for spill slots (pack_alloc, a
// memory-side atomic) right after the block barrier, so the atomic's round trip overlaps the reset
// tail.  The informational header words are not written and the zeroing of the counter is the
// caller's (cf2_xchg_* zeroes a batch's counters in its consume): as little as a block-0 store of
// the header in this kernel slowed even the unpacked env-step from 9.5 to 10.6-11.0 us at 32 768
// envs, and a
// word-interleaved o_k run (one coalesced store per 64 words, ~1000 more instructions) did the same
// (tools/pack_cost_probe.py with ablation builds, gpurun_out/r05r-r05x): the small kernel's env wave
// is sensitive to code anywhere in the kernel.
template <uint32_t OL, uint32_t OD>
__device__ __forceinline__ void pack_epilogue(const PackIO& X, uint32_t n, uint32_t base, uint32_t nvalid,
                                              uint64_t mask, const float* s_obs, const float* s_rrow, uint32_t lane,
                                              uint32_t first) {
    const PackLayout L{n, OL, X.cap};
    uint32_t* pk = X.pk;
    uint32_t* bits = pk + L.bits();
    if (lane == 0) bits[base / 32u] = (uint32_t)mask;
    if (lane == 1 && base + 32u < n) bits[base / 32u + 1u] = (uint32_t)(mask >> 32);
    first = __shfl(first, 0);          // lane 0's pack_alloc, issued right after the block barrier
    if (lane == 0) pk[L.btab() + base / XB_PACK] = first;
    if (lane >= nvalid) return;
    const bool rs = (mask >> lane) & 1ull;
    const float* row = (rs ? s_rrow : s_obs) + lane * OD;
    float* ok = reinterpret_cast<float*>(pk + L.o_slab()) + (size_t)(base + lane) * OL;
#pragma unroll
    for (uint32_t k = 0; k < OL; ++k) ok[k] = row[OL + 4u + k];
    if (!rs) return;
    const uint32_t slot = pack_entry_slot(L, base / XB_PACK, (uint32_t)__popcll(mask & ((1ull << lane) - 1ull)), first);
    if (slot == PACK_DROPPED) return;
    uint32_t* e = pk + L.side() + slot * L.entry();
    e[0] = base + lane;
    float* ef = reinterpret_cast<float*>(e + 1);
#pragma unroll
    for (uint32_t k = 0; k < OL + 4u; ++k) ef[k] = row[k];     // o_0 and A (= A_0)
}

// The small-N kernel's LDS arrays (step_kernel_small declares them; collect_kernel_small carves
// them out of a buffer the policy fragments re-use afterwards)
template <bool NOISE, int SPEC>
struct SmallLds {
    static constexpr int OL = NOISE ? 13 : 17, OD = 2 * (OL + 4);
    // reference-default shape with sensor noise: the helpers also draw the env-step's randomness
    // after its first sub-step (HD_* layout), handed over at an LDS barrier before sub-step 1
    static constexpr bool HD = SPEC == 1 && NOISE;
    // word offsets in a carved buffer (doubles 8-B aligned, rows 16-B aligned)
    // (HD: wave 1 computes the reset pose once and hands it to waves 2-3: POSE_WORDS per env behind
    // the flag word s_mask[2])
    static constexpr uint32_t POSE_WORDS = HD ? 12 : 0;
    static constexpr uint32_t O_OBS = 0, O_RROW = 64 * OD, O_SEED = 128 * OD, O_C2 = O_SEED + SEED_SMALL * 64,
                              O_DRAW = O_C2 + C2_WORDS * 64, O_POSE = O_DRAW + (HD ? HD_WORDS * 64 : 1),
                              O_MASK = O_POSE + (HD ? POSE_WORDS * 64 : 1),
                              O_HJ = (O_MASK + 3 + 1) & ~1u, WORDS = O_HJ + 2 * 6 * HJ_PTS;
};

template <bool NOISE, bool DR, int PHYS, int SPEC>
__device__ __forceinline__ uint64_t small_body(const KParams& P0, const StepIO& io, float* s_obs, float* s_seed,
                                               float* s_c2, float* s_rrow, uint32_t* s_mask, double* s_hjgrid,
                                               float* s_draw, float* s_pose, const PackIO& X = PackIO{}) {
    const KParams P = shape_view<SPEC>(P0);
    using SL = SmallLds<NOISE, SPEC>;
    constexpr int OL = SL::OL;
    constexpr int OD = SL::OD;
    constexpr bool HD = SL::HD;
#ifdef CF2_TIMING
    if (uint64_t* r = timing_row()) {
        if ((threadIdx.x & 63) == 0) {
            const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_ID
            const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);   // XCC_ID
            r[0] = ((uint64_t)xcc << 32) | hw;
            r[1] = __builtin_amdgcn_s_memrealtime();
            r[3] = __builtin_amdgcn_s_memtime();
        }
    }
#endif
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
    const uint32_t base = blockIdx.x * 64u, i = base + lane, gid = P.gid_off + i;
    const bool live = i < P.N;
    if (P.dstb_mode == DSTB_HJ_T) stage_hj_grid(P.tab->hj_grid, s_hjgrid);     // uniform branch
    const Tile T(io.sf, P.N, i);
    // the domain randomisation / disturbance / level draws of the reset: wave 3 (in the
    // reference-default shape wave 1 computes the reset pose for all three helpers meanwhile)
    constexpr uint32_t PARAMS_WAVE = 3u;
    Env H;                         // waves 1-3: the speculative reset (kept across the barrier)
    float held1[10], ng1[9];       // wave 2: first reset sensor call
    HeldNoise hn;                  // waves 2 / 3: the noise of the first / second reset sensor call
    float ngs[9];                  //   and its gyro normals
    uint32_t ctr = 0;
    if (wave != 0 && live) ctr = (uint32_t)bi(T.ld(G_CORE3).z);      // the env's counter (step and reset draws)
    const Keys K = make_keys(P.key0, P.key1);
    const Rng gr{K, ctr, gid, TAG_RESET};
    // the speculative reset's work that needs no reset pose: DR / disturbance / level draws (wave
    // PARAMS_WAVE) and the two reset sensor calls' noise (waves 2, 3), after the draw barrier (all
    // of it before that barrier, in the time the helpers wait there, made the env wave wait at it)
    auto reset_prework = [&]() {
        if (wave == PARAMS_WAVE) {
            const bool need_level = P.need_level || io.level != nullptr;
            H.level = need_level ? T.ld(G_LEVEL).w : P.level_fixed;
            H.level_idx = need_level && P.level_mode != LEVEL_FIXED_T ? bi(T.ld(G_LEVEL_IDX).x) : 0;
            reset_params<DR>(P, H, gr);
        }
        if (NOISE && wave >= 2) held_noise(P, gr, wave == 2 ? 32u : 40u, hn, ngs);
    };
    if (HD && wave != 0) {
        // the env-step's draws after sub-step 0 (step tag, the env's counter), split over the
        // three helper waves; Box-Muller applied where the env-step turns words into normals
        if (live) helper_step_draws(K, ctr, gid, wave, s_draw + lane);
        if (wave == 1 && lane == 0) s_mask[2] = 0u;     // the pose flag (set once the pose is in LDS)
        TSTAMP(10);      // helper: step draws in LDS
        lds_barrier();   // joined by the env wave before its second sub-step (step_env_body)
        TSTAMP(11);
    }
    if (wave == 0) {
        __builtin_amdgcn_s_setprio(3);
        bool do_reset = false;
        ResetSeed rs;
        if (live)
            do_reset = step_env<NOISE, DR, PHYS, true, HD>(P, io, i, s_obs + lane * OD, rs, s_hjgrid, s_draw + lane);
        const uint64_t m = __ballot(do_reset);
        if (lane == 0) { s_mask[0] = (uint32_t)m; s_mask[1] = (uint32_t)(m >> 32); }
        if (do_reset) {
#pragma unroll
            for (int k = 0; k < 3; ++k) { s_seed[k * 64 + lane] = rs.wb[k]; s_seed[(3 + k) * 64 + lane] = rs.bias[k]; }
#pragma unroll
            for (int k = 0; k < 4; ++k) s_seed[(6 + k) * 64 + lane] = rs.ou[k];
        }
    } else if (HD && P.auto_reset && live) {
        // the reset pose computed once, by wave 1 (its step draws are the fewest), and handed to
        // waves 2-3 in LDS while they turn their sensor-call draws into noise (and wave 3 draws the
        // reset's parameters)
        __builtin_amdgcn_s_setprio(0);
        float* row = s_rrow + lane * OD;
        if (wave == 1) {
            reset_kinematics<PHYS>(P, H, gr, gid);
#pragma unroll
            for (int k = 0; k < 4; ++k) { row[OL + k] = H.la[k]; row[2 * OL + 4 + k] = H.la[k]; }
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                s_pose[k * 64 + lane] = H.p[k];
                s_pose[(3 + k) * 64 + lane] = H.v[k];
                s_pose[(6 + k) * 64 + lane] = H.rpy[k];
                s_pose[(9 + k) * 64 + lane] = H.wb[k];
            }
            if (lane == 0) lds_flag_set(s_mask + 2);
        }
        reset_prework();
        if (wave >= 2) {
            lds_flag_wait(s_mask + 2, P.tab);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                H.p[k] = s_pose[k * 64 + lane];
                H.v[k] = s_pose[(3 + k) * 64 + lane];
                H.rpy[k] = s_pose[(6 + k) * 64 + lane];
                H.wb[k] = s_pose[(9 + k) * 64 + lane];
            }
            if (wave == 2) {
                held_combine(H, hn, held1);
#pragma unroll
                for (int k = 0; k < 9; ++k) ng1[k] = ngs[k];
#pragma unroll
                for (int k = 0; k < 10; ++k) row[k] = held1[k];
            } else {
                float held2[10];
                held_combine(H, hn, held2);
#pragma unroll
                for (int k = 0; k < 10; ++k) row[OL + 4 + k] = held2[k];
#pragma unroll
                for (int k = 0; k < 9; ++k) s_c2[k * 64 + lane] = ngs[k];
            }
        }
        TREADY("v"(H.p[0]), "v"(H.K[3]), "v"(H.la[3]));
        TSTAMP(9);   // helper: speculative reset computed
    } else if (!HD && P.auto_reset && live) {
        __builtin_amdgcn_s_setprio(0);
        reset_prework();
        if (wave == 1) {
            reset_kinematics<PHYS>(P, H, gr, gid);
        } else if (wave == 2) {
            reset_kinematics<PHYS>(P, H, gr, gid);
            // the reset observation row [o_0, A_0, o_1, A_1] as far as it does not depend on the
            // finished episode: all of it but the two gyro-LPF triples (o_1's held part: wave 3)
            float* row = s_rrow + lane * OD;
            if (NOISE) {
                held_combine(H, hn, held1);
#pragma unroll
                for (int k = 0; k < 9; ++k) ng1[k] = ngs[k];
#pragma unroll
                for (int k = 0; k < 10; ++k) row[k] = held1[k];
            } else {
                const float o[17] = {H.p[0], H.p[1], H.p[2], H.q[0], H.q[1], H.q[2], H.q[3], H.v[0], H.v[1],
                                     H.v[2], H.wb[0], H.wb[1], H.wb[2], H.la[0], H.la[1], H.la[2], H.la[3]};
#pragma unroll
                for (int k = 0; k < 17; ++k) { row[k] = o[k]; row[OL + 4 + k] = o[k]; }
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) { row[OL + k] = H.la[k]; row[2 * OL + 4 + k] = H.la[k]; }
        } else if (NOISE) {
            Env H2;
            reset_kinematics<PHYS>(P, H2, gr, gid);
            float held2[10];
            held_combine(H2, hn, held2);
            float* row = s_rrow + lane * OD;
#pragma unroll
            for (int k = 0; k < 10; ++k) row[OL + 4 + k] = held2[k];
#pragma unroll
            for (int k = 0; k < 9; ++k) s_c2[k * 64 + lane] = ngs[k];
        }
        TREADY("v"(H.p[0]), "v"(H.K[3]), "v"(H.la[3]));
        TSTAMP(9);   // helper: speculative reset computed
    }
    lds_barrier();
    TSTAMP(4);   // block barrier passed
    const uint64_t mask = ((uint64_t)s_mask[1] << 32) | (uint64_t)s_mask[0];
    const bool mine = wave != 0 && ((mask >> lane) & 1ull);
    uint32_t pk_first = 0u;          // fused pack: the block's first side slot (wave 2, lane 0)
    if (X.pk && wave == 2 && lane == 0 && mask)
        pk_first = pack_alloc(PackLayout{P.N, (uint32_t)OL, X.cap}, X.scratch, (uint32_t)__popcll(mask));
    if (mine) {
        TSTAMP(6);
        if (wave == 1) {
            const float ou[4] = {s_seed[6 * 64 + lane], s_seed[7 * 64 + lane], s_seed[8 * 64 + lane], s_seed[9 * 64 + lane]};
            store_reset_kinematics<PHYS>(P, T, H, ou, ctr);
        } else if (wave == 2) {
            // the reset observation (reset_observe: two sensor calls, then the history row): the
            // gyro-LPF triples of o_0 and o_1 complete the staged row
            Env& E = H;
            float* row = s_rrow + lane * OD;
            if (HD) {
#pragma unroll
                for (int k = 0; k < 4; ++k) E.la[k] = row[OL + k];     // wave 1's, staged in the row
            }
            if (NOISE) {
#pragma unroll
                for (int k = 0; k < 3; ++k) { E.lpf[k] = s_seed[k * 64 + lane]; E.bias[k] = s_seed[(3 + k) * 64 + lane]; }
                float ng2[9];
#pragma unroll
                for (int k = 0; k < 9; ++k) ng2[k] = s_c2[k * 64 + lane];
#pragma unroll
                for (int k = 0; k < 10; ++k) E.held[k] = row[OL + 4 + k];
                gyro_update(P, E, ng1);
#pragma unroll
                for (int k = 0; k < 3; ++k) row[10 + k] = E.lpf[k];
                gyro_update(P, E, ng2);
#pragma unroll
                for (int k = 0; k < 3; ++k) row[OL + 4 + 10 + k] = E.lpf[k];
#pragma unroll
                for (int k = 0; k < 10; ++k) E.obs_prev[k] = E.held[k];
#pragma unroll
                for (int k = 0; k < 3; ++k) E.obs_prev[10 + k] = E.lpf[k];
            } else {
#pragma unroll
                for (int k = 0; k < OL; ++k) E.obs_prev[k] = row[OL + 4 + k];
            }
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                for (int k = 0; k < 4; ++k) E.hact[s2][k] = E.la[k];
            store_reset_history<NOISE>(P, T, E);
            TSTAMP(8);
        }
        if (wave == PARAMS_WAVE) store_reset_params<DR>(P, T, H);
    }
    // the block's obs rows: the chunks of rows whose env did not reset by the env wave (done with
    // its env-step), the chunks touching a reset row by wave 2 once it has completed those rows (its
    // own LDS writes precede its reads; with sensor noise it writes the rows' gyro-LPF triples above).
    // No second barrier: the two sets are disjoint (measured against a block barrier followed by a
    // 256-thread merged write-out: see DESIGN.md section 3).
    const uint32_t nvalid = P.N - base < 64u ? P.N - base : 64u;
    if (wave == 0) write_obs_rows_part<OD>(io.obs + (size_t)base * OD, s_obs, s_rrow, mask, nvalid, lane, false);
    else if (wave == 2) {
        write_obs_rows_part<OD>(io.obs + (size_t)base * OD, s_obs, s_rrow, mask, nvalid, lane, true);
        if (X.pk) pack_epilogue<OL, OD>(X, P.N, base, nvalid, mask, s_obs, s_rrow, lane, pk_first);
    }
    TSTAMP(12);  // rows written
#ifdef CF2_TIMING
    TSTAMP(5);
    if (uint64_t* r = timing_row())
        if ((threadIdx.x & 63) == 0) r[2] = __builtin_amdgcn_s_memrealtime();
#endif
    return mask;
}

template <bool NOISE, bool DR, int PHYS, int SPEC>
__global__ void __launch_bounds__(256, 2) step_kernel_small(KParams P0, StepIO io, PackIO X) {
    using SL = SmallLds<NOISE, SPEC>;
    __shared__ __align__(16) float s_obs[64 * SL::OD];     // the block's obs rows, global layout
    __shared__ float s_seed[SEED_SMALL * 64];              // [word][env]
    __shared__ float s_c2[C2_WORDS * 64];                  // [word][env]
    __shared__ __align__(16) float s_rrow[64 * SL::OD];    // speculative reset observation rows
    __shared__ uint32_t s_mask[3];                         // finished envs (ballot of wave 0), pose flag
    __shared__ double s_hjgrid[6 * HJ_PTS];
    __shared__ float s_draw[SL::HD ? HD_WORDS * 64 : 1];
    __shared__ float s_pose[SL::HD ? SL::POSE_WORDS * 64 : 1];
    (void)small_body<NOISE, DR, PHYS, SPEC>(P0, io, s_obs, s_seed, s_c2, s_rrow, s_mask, s_hjgrid, s_draw, s_pose, X);
}

// The fused collect step at small N (N <= 32 768: the 8-GPU node shard, C2): step_kernel_small's
// env-step (64 envs per block, helper waves), then the policy forward of the block's 64 new
// observations, one 16-row tile per wave.  Alone, the policy kernel at these sizes is a fixed
// cost (weights staging + one tile's dependent chain + a launch: ~15-18 us per step at 4096-32 768
// rows, more than the env-step); here it follows the env-step inside the block.  The final
// observation rows are read from LDS (s_obs, or s_rrow where the env reset), then the block's LDS
// takes the fragments (all but layer 3, as collect_kernel).  Outputs bit-identical to cf2_step +
// cf2_policy_forward.
template <bool NOISE, bool DR, int PHYS, int SPEC>
__global__ void __launch_bounds__(256, 2) collect_kernel_small(KParams P0, StepIO io, PolicyIO pio) {
    static_assert(NOISE, "the fused collect kernel is built for the 34-wide observation");
    using SL = SmallLds<NOISE, SPEC>;
    constexpr int OD = SL::OD;
    using PK = Packed<OD, CF2_POLICY_BF16X3>;
    constexpr uint32_t L3N = PK::O_BIAS - PK::O_L3, POL_WORDS = PK::TOTAL - L3N;
    constexpr uint32_t LDS_WORDS = POL_WORDS > SL::WORDS ? POL_WORDS : SL::WORDS;
    __shared__ __align__(16) float s_mem[LDS_WORDS];
    const uint64_t mask = small_body<NOISE, DR, PHYS, SPEC>(
        P0, io, s_mem + SL::O_OBS, s_mem + SL::O_SEED, s_mem + SL::O_C2, s_mem + SL::O_RROW,
        reinterpret_cast<uint32_t*>(s_mem + SL::O_MASK), reinterpret_cast<double*>(s_mem + SL::O_HJ),
        s_mem + SL::O_DRAW, s_mem + SL::O_POSE);
    // ---- policy phase: wave w takes rows 16 w .. 16 w + 15 of the block (lane l: row 16 w + (l & 15),
    // inputs 8 g .. 8 g + 7 and 32 + g), once wave 2 has completed the reset rows
    lds_barrier();
    const uint32_t tid = threadIdx.x, l = tid & 63u, wv = tid >> 6, r16 = l & 15u;
    const int g = (int)(l >> 4);
    const uint32_t br = 16u * wv + r16, base = blockIdx.x * 64u, row = base + br;
    ObsRegs<OD, CF2_POLICY_BF16X3> X;
    {
        const float* src = (((mask >> br) & 1ull) ? s_mem + SL::O_RROW : s_mem + SL::O_OBS) + br * OD;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float2 v = *reinterpret_cast<const float2*>(src + 8 * g + 2 * q);
            X.x8[0][0][2 * q] = v.x;
            X.x8[0][0][2 * q + 1] = v.y;
        }
        X.x1[0][0] = src[__builtin_elementwise_min(32 + g, OD - 1)];
    }
    __syncthreads();         // every wave holds its rows: the LDS takes the fragments
    constexpr uint32_t NQ4 = POL_WORDS / 4, NQ = (NQ4 + 255u) / 256u;
    float4 stg[NQ];
    {
        const float4* src = reinterpret_cast<const float4*>(pio.w);
#pragma unroll
        for (uint32_t q = 0; q < NQ; ++q) {
            const uint32_t k = __builtin_elementwise_min(tid + q * 256u, NQ4 - 1u);
            stg[q] = src[k < PK::O_L3 / 4 ? k : k + L3N / 4];
        }
    }
    float ep[4];             // this lane's row's sampling noise, drawn while the loads are in flight
    policy_noise(pio.key0, pio.key1, pio.counter, pio.row_offset + row, ep);
    {
        float4* dst = reinterpret_cast<float4*>(s_mem);
#pragma unroll
        for (uint32_t q = 0; q < NQ; ++q)
            if (tid + q * 256u < NQ4) dst[tid + q * 256u] = stg[q];
    }
    __syncthreads();
    PolicyLane<OD, CF2_POLICY_BF16X3> CL;
    policy_lane_init<OD, CF2_POLICY_BF16X3>(s_mem + PK::O_L3, g, CL);
    policy_standardize<OD, CF2_POLICY_BF16X3>(s_mem + PK::O_L3, g, CL, X);
    f4v o[1];
    policy_layers<OD, CF2_POLICY_BF16X3, 0>(s_mem, s_mem + PK::O_L3, pio.w + PK::O_L3, (int)l, X, o);
    if (row < P0.N)
        policy_emit_eps<OD, CF2_POLICY_BF16X3, 0>(o[0], row, g, CL, ep, 1, pio.act, pio.val, pio.logp, nullptr);
}

// One physics sub-step of every env: the physics plugin's step_forward on its own (PyBulletPhysics
// physics.py:91-124, SimplePhysics :130-200, PybulletPhysicsWithAdversary :213-250): apply_action,
// force/torque assembly, drag, rigid-body step and readback; no observation, reward or episode
// counter (cf2_physics_step).  OU normals: Philox block 0 of (rng counter, TAG_PHYS).
template <bool NOISE, bool DR, int PHYS>
__global__ void __launch_bounds__(256) physics_kernel(KParams P, float* __restrict__ sf, const float* __restrict__ act,
                                                      const float* __restrict__ dstb, float dt_override) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.N) return;
    Env E;
    load_env<NOISE, DR, PHYS>(P, sf, i, E, false, /*with_hist=*/false);
    const float4 a4 = reinterpret_cast<const float4*>(act)[i];
    const float a[4] = {a4.x, a4.y, a4.z, a4.w};
    float d[3] = {0.0f, 0.0f, 0.0f};
    if (dstb) {
#pragma unroll
        for (int k = 0; k < 3; ++k) d[k] = dstb[(size_t)i * 3 + k];
    }
    if (dt_override > 0.0f) E.dt = dt_override;
    const Keys K = make_keys(P.key0, P.key1);
    const Rng g{K, E.rng, P.gid_off + i, TAG_PHYS};
    float on[4];
    normals<4>(g, 0, on);
    if (PHYS == PHYS_BULLET_T) {
        if (P.ground_effect) {
            euler_from_quat(E.q, E.rpy);     // drone.rpy of the last readback
            bullet_substep<true>(P, E, a, d, on, E.ep_step == 0 && !E.props_on);
        } else {
            bullet_substep<false>(P, E, a, d, on, E.ep_step == 0 && !E.props_on);
        }
    } else {
#pragma unroll
        for (int k = 0; k < 3; ++k) E.wb[k] = E.w[k];
        simple_substep(P, E, a, on);
    }
    E.props_on = 1;
    E.rng += 1;
    store_core<NOISE, DR, PHYS>(P, sf, i, E);
    const Tile T(sf, P.N, i);
    const int fl = (E.aidx & 15) | (E.halias0 << 4) | (E.halias1 << 5) | (E.la_view << 6) | (E.props_on << 7);
    T.st(G_CORE3, f4(E.w[2], ib(E.ep_step), ib((int)E.rng), ib(fl)));
}

// The fused rollout's auto-resets (rollout_kernel): the block lists its
// finished envs, draws their reset tables block-parallel as step_kernel does, and each env is
// then reset in place by its own lane (its state is in that lane's registers); the reset
// observation goes to row (this lane's LDS row or its global obs row).  Begins and ends with a
// block barrier; s_cnt was zeroed before the first one.
template <bool NOISE, bool DR, int PHYS, uint32_t B, uint32_t C>
__device__ __forceinline__ void rollout_resets(const KParams& P, Env& E, uint32_t base, uint32_t tid, uint32_t i,
                                               bool do_reset, const ResetSeed& rs, uint32_t* s_cnt,
                                               uint32_t* s_list, uint32_t* s_ctr, uint32_t* s_rand, float* row) {
    constexpr int OD = NOISE ? 34 : 42;
    __syncthreads();             // s_cnt initialised
    uint32_t pos = 0;
    const uint64_t m = __ballot(do_reset);
    if (m) {
        const int lane = (int)(threadIdx.x & 63);
        const int leader = __ffsll((unsigned long long)m) - 1;
        if (lane == leader) pos = atomicAdd(s_cnt, (uint32_t)__popcll(m));
        pos = __shfl(pos, leader) + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (do_reset) { s_list[pos] = tid; s_ctr[pos] = rs.ctr; }
    }
    __syncthreads();
    const uint32_t cnt = *s_cnt;
    for (uint32_t c0 = 0; c0 < cnt; c0 += C) {
        const uint32_t nc = cnt - c0 < C ? cnt - c0 : C;
        {
            const Keys Kk = make_keys(P.key0, P.key1);
            for (uint32_t w = tid; w < nc * RESET_SLOTS; w += B) {
                const uint32_t sl = w / nc, e = w - sl * nc, p2 = c0 + e;
                U4 u = philox(Kk, reset_block_of_slot((int)sl), s_ctr[p2], P.gid_off + base + s_list[p2], TAG_RESET);
                if (reset_slot_normal_xy((int)sl)) {
                    float z0, z1;
                    box_muller(u.x, u.y, z0, z1);
                    u.x = __float_as_uint(z0); u.y = __float_as_uint(z1);
                }
                if (reset_slot_normal_zw((int)sl)) {
                    float z2, z3;
                    box_muller(u.z, u.w, z2, z3);
                    u.z = __float_as_uint(z2); u.w = __float_as_uint(z3);
                }
                uint32_t* q = s_rand + sl * 4 * C + e;
                q[0] = u.x; q[C] = u.y; q[2 * C] = u.z; q[3 * C] = u.w;
            }
        }
        __syncthreads();
        if (do_reset && pos >= c0 && pos < c0 + nc) {
            // reset_env keeps what a reset inherits from the finished episode (stale body rates,
            // gyro bias, OU state, level) from E itself
            float o[OD];
            const TableRng tg{s_rand + (pos - c0), C};
            reset_env<NOISE, DR, PHYS, /*TAB=*/true>(P, E, tg, P.gid_off + i, o);
#pragma unroll
            for (int q = 0; q < OD; q += 2) *reinterpret_cast<float2*>(row + q) = make_float2(o[q], o[q + 1]);
        }
        __syncthreads();         // the next chunk reuses s_rand
    }
}

// Fused K-step rollout (cf2_rollout): the env state is loaded once, stays in registers for K
// env-steps and is stored once.  Step k reads its actions at act + k * act_stride and writes its
// outputs into the k-th [N, ...] slab of each output (obs, rew, done, trunc, cost, level,
// final_obs), i.e. exactly what K cf2_step calls would write.  Auto-reset: the block lists its
// finished envs and draws their reset tables block-parallel as step_kernel does, but each env is
// then reset in place by its own lane (its state is in that lane's registers); per env-step HBM
// traffic is the actions and the outputs only (~170 B instead of ~765 B).
// 2 waves per SIMD: the whole state stays live across the loop (~270 registers at peak).  The 20
// Philox round keys in SGPRs make it spill 28 B/lane of VGPRs (7 registers); re-deriving them per
// Philox call removes every VGPR spill but was slower on MI355X (K = 32 per env-step: 27.9 -> 30.0
// us at 262 144 envs, 8.5 -> 10.1 us at 4096): the SALU adds sit in each Philox chain, the spills
// do not.
constexpr uint32_t ROLL_MIN_WAVES = 2;
template <bool NOISE, bool DR, int PHYS, int SPEC>
__global__ void __launch_bounds__(STEP_BLOCK, ROLL_MIN_WAVES) rollout_kernel(KParams P0, StepIO io0, uint32_t K,
                                                                          uint32_t act_stride) {
    const KParams P = shape_view<SPEC>(P0);
    constexpr int OD = NOISE ? 34 : 42;
    constexpr uint32_t B = STEP_BLOCK, EPB = STEP_BLOCK;
    constexpr uint32_t C = RESET_CHUNK;
    __shared__ __align__(16) float s_obs[B * OD];
    __shared__ uint32_t s_list[B];
    __shared__ uint32_t s_ctr[B];                       // rng counter of each listed env's reset
    __shared__ uint32_t s_rand[RESET_SLOTS * 4 * C];
    __shared__ uint32_t s_cnt;
    __shared__ double s_hjgrid[6 * HJ_PTS];
    const uint32_t tid = threadIdx.x, base = blockIdx.x * EPB, i = base + tid;
    if (P.dstb_mode == DSTB_HJ_T) stage_hj_grid(P.tab->hj_grid, s_hjgrid);     // uniform branch
    const bool live = tid < EPB && i < P.N;
    const bool need_level = P.need_level || io0.level != nullptr;
    Env E;
    if (live) load_env<NOISE, DR, PHYS>(P, io0.sf, i, E, need_level, /*with_hist=*/true);
    const size_t n = P0.out_stride;              // rows per output slab (the whole population)
    float* obs_row = s_obs + tid * OD;
    for (uint32_t k = 0; k < K; ++k) {
        if (tid == 0) s_cnt = 0;     // every reader of the previous step passed its last barrier
        const StepIO I0 = late_io(io0);
        StepIO io = I0;
        io.act = I0.act + (size_t)k * act_stride;
        io.rew = I0.rew + (size_t)k * n;
        io.done = I0.done + (size_t)k * n;
        if (I0.trunc) io.trunc = I0.trunc + (size_t)k * n;
        if (I0.cost) io.cost = I0.cost + (size_t)k * n;
        if (I0.level) io.level = I0.level + (size_t)k * n;
        if (I0.final_obs) io.final_obs = I0.final_obs + (size_t)k * n * OD;
        bool do_reset = false;
        ResetSeed rs;
        if (live) do_reset = step_env_body<NOISE, DR, PHYS, false, false, false, 0, false, true>(P, io, i, E, obs_row, rs, s_hjgrid);
        rollout_resets<NOISE, DR, PHYS, B, C>(P, E, base, tid, i, do_reset, rs, &s_cnt, s_list, s_ctr, s_rand, obs_row);
        // coalesced write of the block's obs rows into step k's slab
        write_obs_rows<EPB, OD, B>(io0.obs + (size_t)k * n * OD + (size_t)base * OD, s_obs,
                                   P.N - base < EPB ? P.N - base : EPB, tid);
        __syncthreads();             // the write-out read s_obs before the next step's rows
    }
    if (live) store_env<NOISE, DR, PHYS>(P, io0.sf, i, E, /*params_dirty=*/true);
}

// Small-N fused rollout (N <= 32 768): 64 envs per 256-thread block, their state in wave 0's
// registers for all K steps, as rollout_kernel<.., 64>.  Waves 1-3 do for the rollout what they do
// for one step in step_kernel_small: while wave 0 steps, they draw the step's randomness after
// sub-step 0 (reference-default shape with sensor noise, the HD_* layout) and compute every env's
// potential auto-reset speculatively (its draws are keyed by the env's RNG counter, which advances
// by one per env-step), leaving the parts that do not depend on the finished episode in LDS
// records: the reset pose, velocities, motor state, latency ring (RK_*), the domain randomisation,
// disturbance and level (RP_*), and the two reset sensor calls' held measurements and gyro normals
// (RO_*).  After one LDS barrier wave 0 only copies a record into a finishing env's registers and
// runs the two gyro updates that need the finished episode's body rates and gyro bias.  Per step:
// barrier A (wave 0 in sub-step 1 with HD, else at the top of the step; helpers write step k's
// records only after it, so wave 0 has read step k-1's) and barrier B (records and the finished
// envs' ballot in LDS).
enum { RK_P = 0, RK_Q = 3, RK_V = 7, RK_W = 10, RK_RPY = 13, RK_WB = 16, RK_X = 19, RK_ABUF = 23, RK_LA = 39,
       RK_WORDS = 43 };
enum { RP_DT = 0, RP_M = 1, RP_J = 2, RP_K0 = 5, RP_K1 = 6, RP_B = 7, RP_K = 11, RP_DSTB = 15, RP_LEVEL = 18,
       RP_LEVEL_IDX = 19, RP_WORDS = 20 };
enum { RO_HELD1 = 0, RO_NG1 = 10, RO_HELD2 = 19, RO_NG2 = 29, RO_WORDS = 38 };

// LDS records of one 64-env group of the small-N fused rollouts ([word][env] columns)
struct SmallRollLds {
    float* obs;          // [64][OD] the group's obs rows
    float* kin;          // [RK_WORDS][64]
    float* par;          // [RP_WORDS][64]
    float* ho;           // [RO_WORDS][64] (sensor noise only)
    float* draw;         // [HD_WORDS][64] (HD only)
    uint32_t* mask;      // [3] the group's finished envs (ballot of its env wave), the pose flag
};

// The env wave's part of one step of the small-N fused rollouts: the env-step (barrier A_k inside
// it with HD, else at the top), the ballot, barrier B_k, and a finishing env's reset copied from
// the helpers' records into its registers, its reset observation row into L.obs.
template <bool NOISE, bool DR, int PHYS, int SPEC>
__device__ __forceinline__ void small_roll_env_step(const KParams& P, const StepIO& io, uint32_t i, uint32_t lane,
                                                    bool live, Env& E, const SmallRollLds& L, const double* s_hjgrid) {
    constexpr int OL = NOISE ? 13 : 17;
    constexpr int OD = 2 * (OL + 4);
    constexpr bool HD = SPEC == 1 && NOISE;
    float* obs_row = L.obs + lane * OD;
    if (!HD) lds_barrier();                  // A_k (HD: inside the env-step, before sub-step 1)
    bool do_reset = false;
    ResetSeed rs;
    if (live)
        do_reset = step_env_body<NOISE, DR, PHYS, false, false, HD, 0, false, true>(P, io, i, E, obs_row, rs, s_hjgrid,
                                                                                    L.draw + lane);
    const uint64_t m = __ballot(do_reset);
    if (lane == 0) { L.mask[0] = (uint32_t)m; L.mask[1] = (uint32_t)(m >> 32); }
    lds_barrier();                           // B_k: the helpers' records of step k are in LDS
    if (do_reset) {
        const float stale[3] = {rs.wb[0], rs.wb[1], rs.wb[2]};   // the gyro LPF seed
        const float* kin = L.kin + lane;
        const float* par = L.par + lane;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            E.p[c] = kin[(RK_P + c) * 64]; E.v[c] = kin[(RK_V + c) * 64]; E.w[c] = kin[(RK_W + c) * 64];
            E.rpy[c] = kin[(RK_RPY + c) * 64]; E.wb[c] = kin[(RK_WB + c) * 64];
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            E.q[c] = kin[(RK_Q + c) * 64]; E.x[c] = kin[(RK_X + c) * 64]; E.xl[c] = 0.0f;
            E.la[c] = kin[(RK_LA + c) * 64];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) E.abuf[r][c] = r < P.buf_size ? kin[(RK_ABUF + 4 * r + c) * 64] : 0.0f;
        E.ep_step = 0; E.aidx = 0; E.props_on = 0; E.la_view = 1;
        E.dt = par[RP_DT * 64]; E.m = par[RP_M * 64];
#pragma unroll
        for (int c = 0; c < 3; ++c) { E.J[c] = par[(RP_J + c) * 64]; E.dstb[c] = par[(RP_DSTB + c) * 64]; }
        E.k0 = par[RP_K0 * 64]; E.k1 = par[RP_K1 * 64];
#pragma unroll
        for (int c = 0; c < 4; ++c) { E.B[c] = par[(RP_B + c) * 64]; E.K[c] = par[(RP_K + c) * 64]; }
        E.level = par[RP_LEVEL * 64];
        E.level_idx = bi(par[RP_LEVEL_IDX * 64]);
        E.gust_left = 0;
        // the reset observation (reset_observe): two sensor calls, then the history row
        float o0[17], o1[17];
        if (NOISE) {
            const float* ho = L.ho + lane;
            float ng1[9], ng2[9];
#pragma unroll
            for (int c = 0; c < 9; ++c) { ng1[c] = ho[(RO_NG1 + c) * 64]; ng2[c] = ho[(RO_NG2 + c) * 64]; }
#pragma unroll
            for (int c = 0; c < 3; ++c) E.lpf[c] = stale[c];
#pragma unroll
            for (int c = 0; c < 10; ++c) { o0[c] = ho[(RO_HELD1 + c) * 64]; o1[c] = ho[(RO_HELD2 + c) * 64]; }
#pragma unroll
            for (int c = 0; c < 10; ++c) E.held[c] = o1[c];
            gyro_update(P, E, ng1);
#pragma unroll
            for (int c = 0; c < 3; ++c) o0[10 + c] = E.lpf[c];
            gyro_update(P, E, ng2);
#pragma unroll
            for (int c = 0; c < 3; ++c) o1[10 + c] = E.lpf[c];
        } else {
            const float o[17] = {E.p[0], E.p[1], E.p[2], E.q[0], E.q[1], E.q[2], E.q[3], E.v[0], E.v[1],
                                 E.v[2], E.wb[0], E.wb[1], E.wb[2], E.la[0], E.la[1], E.la[2], E.la[3]};
#pragma unroll
            for (int c = 0; c < 17; ++c) { o0[c] = o[c]; o1[c] = o[c]; }
        }
        float row[OD];
#pragma unroll
        for (int c = 0; c < OL; ++c) { row[c] = o0[c]; row[OL + 4 + c] = o1[c]; E.obs_prev[c] = o1[c]; }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            row[OL + c] = E.la[c]; row[2 * OL + 4 + c] = E.la[c];
            E.hact[0][c] = E.la[c]; E.hact[1][c] = E.la[c];
        }
        E.halias0 = E.halias1 = 1;
#pragma unroll
        for (int c = 0; c < OD; c += 2) *reinterpret_cast<float2*>(obs_row + c) = make_float2(row[c], row[c + 1]);
    }
}

// A helper wave's part of one step (wave 1-3 of a group): the HD draws of step k, barrier A_k, the
// speculative reset of every env of the group into the LDS records, barrier B_k, and the level a
// finishing env's new episode keeps.  ctr: the env's RNG counter at step k.
template <bool NOISE, bool DR, int PHYS, int SPEC>
__device__ __forceinline__ void small_roll_helper_step(const KParams& P, const Keys& Kh, uint32_t ctr, uint32_t gid,
                                                       uint32_t wave, uint32_t lane, bool live, float& lvl,
                                                       int& lvl_idx, const SmallRollLds& L) {
    constexpr bool HD = SPEC == 1 && NOISE;
    constexpr uint32_t PARAMS_WAVE = 3u;
    if (HD) {
        if (live) helper_step_draws(Kh, ctr, gid, wave, L.draw + lane);
    }
    if (NOISE && wave == 1 && lane == 0) L.mask[2] = 0u;     // the pose flag of step k
    lds_barrier();                               // A_k
    Env H;
    if (P.auto_reset && live) {
        const Rng gr{Kh, ctr, gid, TAG_RESET};
        auto params = [&]() {
            H.level = lvl;
            H.level_idx = lvl_idx;
            reset_params<DR, true>(P, H, gr);
            float* par = L.par + lane;
            par[RP_DT * 64] = H.dt; par[RP_M * 64] = H.m;
#pragma unroll
            for (int c = 0; c < 3; ++c) { par[(RP_J + c) * 64] = H.J[c]; par[(RP_DSTB + c) * 64] = H.dstb[c]; }
            par[RP_K0 * 64] = H.k0; par[RP_K1 * 64] = H.k1;
#pragma unroll
            for (int c = 0; c < 4; ++c) { par[(RP_B + c) * 64] = H.B[c]; par[(RP_K + c) * 64] = H.K[c]; }
            par[RP_LEVEL * 64] = H.level;
            par[RP_LEVEL_IDX * 64] = ib(H.level_idx);
        };
        // the reset pose once, by wave 1, into the kinematics record; with sensor noise waves 2-3
        // read its position, velocity and attitude from there once wave 1 has set the flag (they
        // draw their sensor-call noise, and wave 3 the reset's parameters, meanwhile)
        if (wave == 1) {
            reset_kinematics<PHYS, true>(P, H, gr, gid);
            float* kin = L.kin + lane;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                kin[(RK_P + c) * 64] = H.p[c]; kin[(RK_V + c) * 64] = H.v[c]; kin[(RK_W + c) * 64] = H.w[c];
                kin[(RK_RPY + c) * 64] = H.rpy[c]; kin[(RK_WB + c) * 64] = H.wb[c];
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                kin[(RK_Q + c) * 64] = H.q[c]; kin[(RK_X + c) * 64] = H.x[c]; kin[(RK_LA + c) * 64] = H.la[c];
            }
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    if (r < P.buf_size) kin[(RK_ABUF + 4 * r + c) * 64] = H.abuf[r][c];
            if (NOISE && lane == 0) lds_flag_set(L.mask + 2);
        } else if (NOISE) {
            HeldNoise hn;
            float ngs[9];
            held_noise(P, gr, wave == 2 ? 32u : 40u, hn, ngs);
            if (wave == PARAMS_WAVE) params();
            lds_flag_wait(L.mask + 2, P.tab);
            const float* kin = L.kin + lane;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                H.p[c] = kin[(RK_P + c) * 64]; H.v[c] = kin[(RK_V + c) * 64]; H.rpy[c] = kin[(RK_RPY + c) * 64];
            }
            float held[10];
            held_combine(H, hn, held);
            float* ho = L.ho + lane;
            const int hb = wave == 2 ? RO_HELD1 : RO_HELD2, nb = wave == 2 ? RO_NG1 : RO_NG2;
#pragma unroll
            for (int c = 0; c < 10; ++c) ho[(hb + c) * 64] = held[c];
#pragma unroll
            for (int c = 0; c < 9; ++c) ho[(nb + c) * 64] = ngs[c];
        }
        if (!NOISE && wave == PARAMS_WAVE) params();
    }
    lds_barrier();                               // B_k
    if (P.auto_reset && live && wave == PARAMS_WAVE) {
        const uint64_t mask = ((uint64_t)L.mask[1] << 32) | (uint64_t)L.mask[0];
        if ((mask >> lane) & 1ull) { lvl = H.level; lvl_idx = H.level_idx; }   // the new episode's level
    }
}

template <bool NOISE, bool DR, int PHYS, int SPEC>
__global__ void __launch_bounds__(256, 2) rollout_kernel_small(KParams P0, StepIO io0, uint32_t K, uint32_t act_stride) {
    const KParams P = shape_view<SPEC>(P0);
    constexpr int OL = NOISE ? 13 : 17;
    constexpr int OD = 2 * (OL + 4);
    constexpr bool HD = SPEC == 1 && NOISE;
    constexpr uint32_t PARAMS_WAVE = 3u;          // as small_roll_helper_step's
    __shared__ __align__(16) float s_obs[64 * OD];
    __shared__ float s_kin[RK_WORDS * 64];                 // [word][env]
    __shared__ float s_par[RP_WORDS * 64];
    __shared__ float s_ho[NOISE ? RO_WORDS * 64 : 1];
    __shared__ float s_draw[HD ? HD_WORDS * 64 : 1];
    __shared__ uint32_t s_mask[3];
    __shared__ double s_hjgrid[6 * HJ_PTS];
    const SmallRollLds L{s_obs, s_kin, s_par, s_ho, s_draw, s_mask};
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
    const uint32_t base = blockIdx.x * 64u, i = base + lane, gid = P.gid_off + i;
    const bool live = i < P.N;
    const bool need_level = P.need_level || io0.level != nullptr;
    if (P.dstb_mode == DSTB_HJ_T) stage_hj_grid(P.tab->hj_grid, s_hjgrid);     // uniform branch
    const size_t n = P0.out_stride;              // rows per output slab (the whole population)
    if (wave == 0) {
        __builtin_amdgcn_s_setprio(3);
        Env E;
        if (live) load_env<NOISE, DR, PHYS>(P, io0.sf, i, E, need_level, /*with_hist=*/true);
        for (uint32_t k = 0; k < K; ++k) {
            const StepIO I0 = late_io(io0);
            StepIO io = I0;
            io.act = I0.act + (size_t)k * act_stride;
            io.rew = I0.rew + (size_t)k * n;
            io.done = I0.done + (size_t)k * n;
            if (I0.trunc) io.trunc = I0.trunc + (size_t)k * n;
            if (I0.cost) io.cost = I0.cost + (size_t)k * n;
            if (I0.level) io.level = I0.level + (size_t)k * n;
            if (I0.final_obs) io.final_obs = I0.final_obs + (size_t)k * n * OD;
            small_roll_env_step<NOISE, DR, PHYS, SPEC>(P, io, i, lane, live, E, L, s_hjgrid);
            // this wave's 64 rows, written by this wave only: its LDS writes land before its reads
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            write_obs_rows<64u, OD, 64u>(io0.obs + (size_t)k * n * OD + (size_t)base * OD, s_obs,
                                         P.N - base < 64u ? P.N - base : 64u, lane);
        }
        if (live) store_env<NOISE, DR, PHYS>(P, io0.sf, i, E, /*params_dirty=*/true);
        return;
    }
    // helper waves 1-3
    __builtin_amdgcn_s_setprio(0);
    uint32_t ctr = 0;
    float lvl = 0.0f;
    int lvl_idx = 0;
    if (live) {
        const Tile T(io0.sf, P.N, i);
        ctr = (uint32_t)bi(T.ld(G_CORE3).z);
        if (wave == PARAMS_WAVE) {
            lvl = need_level ? T.ld(G_LEVEL).w : P.level_fixed;
            lvl_idx = need_level && P.level_mode != LEVEL_FIXED_T ? bi(T.ld(G_LEVEL_IDX).x) : 0;
        }
    }
    const Keys Kh = make_keys(P.key0, P.key1);
    for (uint32_t k = 0; k < K; ++k, ++ctr)
        small_roll_helper_step<NOISE, DR, PHYS, SPEC>(P, Kh, ctr, gid, wave, lane, live, lvl, lvl_idx, L);
}

// The collect loop in one launch at small N (N <= 32 768: the 8-GPU node shard, C2).  A 512-thread
// block holds two 64-env groups, each run as rollout_kernel_small runs its block (wave 0 of the
// group steps its envs with the state in registers, waves 1-3 compute the potential resets and the
// step's draws), and after each env-step all 8 waves run the policy forward, one 16-row tile each,
// on the block's 128 new observations (still in LDS), whose actions the next env-step reads.
// Per step: barriers A_k, B_k (rollout_kernel_small's), P_k (every reset row is in LDS) and Q_k
// (the step's actions are visible to the env waves).  LDS: the fragments (60.8 KB, staged once)
// and two groups' records (2 x 46.6 KB): one block per CU, 8 waves, as two blocks of
// step_kernel_small; 32 768 envs are one residency round of 256 blocks.  Outputs bit-identical
// to K cf2_collect_step launches (the same device code for both halves).
constexpr uint32_t CROLL_SMALL_BLOCK = 512;
template <bool NOISE, bool DR, int PHYS, int SPEC>
__global__ void __launch_bounds__(CROLL_SMALL_BLOCK, 1) collect_rollout_kernel_small(KParams P0, StepIO io0,
                                                                                    PolicyIO pio, uint32_t K) {
    static_assert(NOISE && SPEC == 1, "the fused collect kernels are built for the reference-default shape with noise");
    const KParams P = shape_view<SPEC>(P0);
    constexpr int OD = 34;
    constexpr uint32_t PARAMS_WAVE = 3u;          // as small_roll_helper_step's
    using PK = Packed<OD, CF2_POLICY_BF16X3>;
    static_assert(PK::TOTAL % 4 == 0, "float4 staging");
    __shared__ __align__(16) float s_frag[PK::TOTAL];
    __shared__ __align__(16) float s_obs[2][64 * OD];
    __shared__ float s_kin[2][RK_WORDS * 64];
    __shared__ float s_par[2][RP_WORDS * 64];
    __shared__ float s_ho[2][RO_WORDS * 64];
    __shared__ float s_draw[2][HD_WORDS * 64];
    __shared__ uint32_t s_mask[2][3];
    __shared__ double s_hjgrid[6 * HJ_PTS];
    const uint32_t tid = threadIdx.x, wv = tid >> 6, grp = wv >> 2, wave = wv & 3u, lane = tid & 63u;
    const uint32_t base = blockIdx.x * 128u, gbase = base + 64u * grp, i = gbase + lane, gid = P.gid_off + i;
    const bool live = i < P.N;
    const SmallRollLds L{s_obs[grp], s_kin[grp], s_par[grp], s_ho[grp], s_draw[grp], s_mask[grp]};
    if (P.dstb_mode == DSTB_HJ_T) stage_hj_grid(P.tab->hj_grid, s_hjgrid);     // uniform branch
    {
        const float4* src = reinterpret_cast<const float4*>(pio.w);
        float4* dst = reinterpret_cast<float4*>(s_frag);
        for (uint32_t q = tid; q < PK::TOTAL / 4; q += CROLL_SMALL_BLOCK) dst[q] = src[q];
    }
    __syncthreads();                             // the fragments are in LDS
    const size_t n = P0.out_stride;              // rows per output slab (the whole population)
    const uint32_t nrows = P.N - base < 128u ? P.N - base : 128u;    // rows of this block (> 0)
    // policy tile of this wave: block rows 16 wv .. 16 wv + 15 (group wv / 4, its rows 16 (wv & 3) ..)
    const uint32_t r16 = lane & 15u, trow = 16u * wv + r16;
    const int g = (int)(lane >> 4);
    const float* trow_lds = &s_obs[wv >> 2][(16u * (wv & 3u) + r16) * OD];
    auto policy_tile = [&](uint32_t k) {
        float ep[4];
        policy_noise(pio.key0, pio.key1, pio.counter + k, pio.row_offset + base + trow, ep);   // lanes 0-15 use it
        PolicyLane<OD, CF2_POLICY_BF16X3> CL;
        policy_lane_init<OD, CF2_POLICY_BF16X3>(s_frag + PK::O_BIAS, g, CL);
        ObsRegs<OD, CF2_POLICY_BF16X3, 1> Xc;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float2 v = *reinterpret_cast<const float2*>(trow_lds + 8 * g + 2 * q);
            Xc.x8[0][0][2 * q] = v.x;
            Xc.x8[0][0][2 * q + 1] = v.y;
        }
        Xc.x1[0][0] = trow_lds[__builtin_elementwise_min(32 + g, OD - 1)];
        policy_standardize<OD, CF2_POLICY_BF16X3, 1>(s_frag + PK::O_BIAS, g, CL, Xc);
        f4v o[1];
        policy_layers<OD, CF2_POLICY_BF16X3, 0, 1>(s_frag, s_frag + PK::O_BIAS, s_frag + PK::O_L3, (int)lane, Xc, o);
        if (trow < nrows)
            policy_emit_eps<OD, CF2_POLICY_BF16X3, 0>(o[0], base + trow, g, CL, ep, 1,
                                                      pio.act + (size_t)(k + 1) * n * 4, pio.val + (size_t)(k + 1) * n,
                                                      pio.logp + (size_t)(k + 1) * n, nullptr);
    };
    // the block's rows of step k into its obs slab: this wave's 16 rows (read from LDS after P_k)
    auto write_rows = [&](uint32_t k) {
        const uint32_t r0 = 16u * wv;
        if (r0 >= nrows) return;
        const uint32_t nr = nrows - r0 < 16u ? nrows - r0 : 16u;
        const float2* src = reinterpret_cast<const float2*>(&s_obs[wv >> 2][16u * (wv & 3u) * OD]);
        float2* dst = reinterpret_cast<float2*>(io0.obs + (size_t)k * n * OD + (size_t)(base + r0) * OD);
        for (uint32_t q = lane; q < nr * (OD / 2); q += 64u) dst[q] = src[q];
    };
    if (wave == 0) {
        __builtin_amdgcn_s_setprio(3);
        Env E;
        if (live) load_env<NOISE, DR, PHYS>(P, io0.sf, i, E, P.need_level, /*with_hist=*/true);
        for (uint32_t k = 0; k < K; ++k) {
            const StepIO I0 = late_io(io0);
            StepIO io = I0;
            io.act = pio.act + (size_t)k * n * 4;
            io.rew = I0.rew + (size_t)k * n;
            io.done = I0.done + (size_t)k * n;
            if (I0.trunc) io.trunc = I0.trunc + (size_t)k * n;
            if (I0.final_obs) io.final_obs = I0.final_obs + (size_t)k * n * OD;
            small_roll_env_step<NOISE, DR, PHYS, SPEC>(P, io, i, lane, live, E, L, s_hjgrid);
            lds_barrier();                       // P_k: every row of the block is in LDS
            write_rows(k);
            policy_tile(k);
            __syncthreads();                     // Q_k: step k + 1's actions are visible, s_obs is free
        }
        if (live) store_env<NOISE, DR, PHYS>(P, io0.sf, i, E, /*params_dirty=*/true);
        return;
    }
    // helper waves 1-3 of the group
    __builtin_amdgcn_s_setprio(0);
    uint32_t ctr = 0;
    float lvl = 0.0f;
    int lvl_idx = 0;
    if (live) {
        const Tile T(io0.sf, P.N, i);
        ctr = (uint32_t)bi(T.ld(G_CORE3).z);
        if (wave == PARAMS_WAVE) {
            lvl = P.need_level ? T.ld(G_LEVEL).w : P.level_fixed;
            lvl_idx = P.need_level && P.level_mode != LEVEL_FIXED_T ? bi(T.ld(G_LEVEL_IDX).x) : 0;
        }
    }
    const Keys Kh = make_keys(P.key0, P.key1);
    for (uint32_t k = 0; k < K; ++k, ++ctr) {
        small_roll_helper_step<NOISE, DR, PHYS, SPEC>(P, Kh, ctr, gid, wave, lane, live, lvl, lvl_idx, L);
        lds_barrier();                           // P_k
        write_rows(k);
        policy_tile(k);
        __syncthreads();                         // Q_k
    }
}

template <bool NOISE, bool DR, int PHYS, int SPEC>
__global__ void __launch_bounds__(256) reset_kernel(KParams P0, float* __restrict__ sf,
                                                    const uint8_t* __restrict__ mask, float* __restrict__ obs) {
    const KParams P = shape_view<SPEC>(P0);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.N) return;
    if (mask && !mask[i]) return;
    reset_one<NOISE, DR, PHYS>(P, sf, i, obs);
}

// initial (pre-reset) state: AgentBase defaults, nominal params
__global__ void init_kernel(KParams P, float* __restrict__ sf) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.N) return;
    const Tile T(sf, P.N, i);
    const F4 z = f4(0.0f, 0.0f, 0.0f, 0.0f);
    for (int g = 0; g < NG; ++g) T.st(g, z);
    T.st(0, f4(0.0f, 0.0f, 1.0f, 0.0f));                 // pos (0, 0, 1), quat x
    T.st(1, f4(0.0f, 0.0f, 1.0f, 0.0f));                 // quat (.., w = 1), vel x
    T.st(G_PARAM, f4(P.time_step, P.mass, P.ixx, P.iyy));
    T.st(G_PARAM + 1, f4(P.izz, P.ft0, P.ft1, P.B));
    T.st(G_PARAM + 2, f4(P.B, P.B, P.B, P.K));
    float level = P.level_fixed;
    int li = 0;
    if (P.level_mode == LEVEL_BOLTZMANN_T) {
        // construction-time Boltzmann() draw (hover_free.py:488), rng counter 0xFFFFFFFF
        const Keys K = make_keys(P.key0, P.key1);
        const Rng g{K, 0xFFFFFFFFu, P.gid_off + i, TAG_RESET};
        const U4 u = g.block(0);
        li = boltzmann_index(P, u01(u.x));
        level = P.tab->level_values[li];
    }
    T.st(G_LEVEL, f4(P.K, P.K, P.K, level));
    T.st(G_LEVEL_IDX, f4(ib(li), 0.0f, 0.0f, 0.0f));
}

// public snapshot field -> internal slot (cf2sim_internal.h)
// -1: motor A[j] (derived), -2: not stored in this configuration (the gyro LPF without noise)
__device__ __forceinline__ int pub_float_slot(int f, bool noise) {
    if (f < F_RPY) return f;                              // pos, quat, vel, omega: same slots
    if (f < F_MOTOR) return S_RPY + (f - F_RPY);
    if (f < F_LPF) return f;                              // motor, ou, abuf, bias: same slots
    if (f < F_HELD) return noise ? S_LPF + (f - F_LPF) : -2;
    if (f < F_OBS_PREV) return S_HELD + (f - F_HELD);
    if (f < F_HIST_ACT) return S_OBSP + (f - F_OBS_PREV);
    if (f < F_PARAM) return S_HACT + (f - F_HIST_ACT);
    if (f < F_DSTB) {                                     // dt m J k0 k1 | A[4] | B[4] K[4]
        const int k = f - F_PARAM;
        if (k < 7) return S_PARAM + k;
        if (k < 11) return -1;                            // A = 1 - B: derived, not stored
        return S_PARAM + k - 4;
    }
    if (f < F_LEVEL) return S_DSTB + (f - F_DSTB);
    if (f == F_LEVEL) return S_LEVEL;
    return S_MOTOR_LO + (f - F_MOTOR_LO);
}
__device__ __forceinline__ int pub_int_slot(int f) {
    switch (f) {
    case I_EP_STEP: return S_EP;
    case I_RNG: return S_RNG;
    case I_FLAGS: return S_FLAGS;
    case I_LEVEL: return S_LEVEL_IDX;
    default: return S_GUST;
    }
}
__device__ __forceinline__ size_t slot_index(uint32_t i, int slot) {     // in floats
    return (size_t)(i >> 6) * (NG * 256) + (size_t)(slot >> 2) * 256 + (i & 63u) * 4 + (slot & 3);
}
__global__ void state_convert_kernel(uint32_t N, float* __restrict__ sf, float* __restrict__ pf,
                                     int32_t* __restrict__ pi, int to_public, int noise) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    for (int f = 0; f < NF; ++f) {
        const int slot = pub_float_slot(f, noise != 0);
        if (slot == -2) {    // not stored: exported as 0, ignored on import
            if (to_public) pf[(size_t)f * N + i] = 0.0f;
            continue;
        }
        if (slot < 0) {      // motor A[j]: exported as 1 - B[j], ignored on import
            if (to_public) pf[(size_t)f * N + i] = 1.0f - sf[slot_index(i, pub_float_slot(f + 4, noise != 0))];
            continue;
        }
        float* in = sf + slot_index(i, slot);
        if (to_public) pf[(size_t)f * N + i] = *in;
        else *in = pf[(size_t)f * N + i];
    }
    for (int f = 0; f < NI; ++f) {
        float* in = sf + slot_index(i, pub_int_slot(f));
        if (to_public) pi[(size_t)f * N + i] = __float_as_int(*in);
        else *in = __int_as_float(pi[(size_t)f * N + i]);
    }
}

// the grid nodes arrive by value in the kernarg segment (720 B): the stand-alone call needs no
// device table, allocation or host synchronisation
// one thread per grid node: the sign bits hj_signs would compute for any state nearest to it
__global__ void __launch_bounds__(256) hj_sign_table_kernel(const float* __restrict__ V, uint32_t total,
                                                            uint8_t* __restrict__ bits) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= total) return;
    const uint32_t t = k / (uint32_t)HJ_TABLE, c = k - t * (uint32_t)HJ_TABLE;
    int idx[6];
    uint32_t r = c;
#pragma unroll
    for (int d = 5; d >= 0; --d) { idx[d] = (int)(r % HJ_PTS); r /= HJ_PTS; }
    bits[k] = (uint8_t)hj_node_bits(V + (size_t)t * HJ_TABLE, (int)c, idx);
}

__global__ void hj_kernel(HjGrid G, double3 umax, const float* __restrict__ V, const float* __restrict__ states,
                          uint32_t n, float level, float* __restrict__ dstb, float* __restrict__ uopt) {
    __shared__ double s_grid[6 * HJ_PTS];
    stage_hj_grid(G.p, s_grid);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double st[6];
#pragma unroll
    for (int d = 0; d < 6; ++d) st[d] = (double)states[(size_t)i * 6 + d];
    const unsigned bits = hj_signs(V, st, s_grid);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double um = k == 0 ? umax.x : (k == 1 ? umax.y : umax.z);
        const double dm = (double)level * um;
        dstb[(size_t)i * 3 + k] = (float)((bits >> k) & 1u ? -dm : dm);
        if (uopt) uopt[(size_t)i * 3 + k] = (float)((bits >> k) & 1u ? -um : um);
    }
}

// ------------------------------------------------------------------------------------
// host-side launch table
// ------------------------------------------------------------------------------------
// Blocks resident at once (CUs x blocks per CU at the kernel's VGPR / LDS use) of the large-N
// kernels of this configuration, queried once per context at cf2_create for the context's device
// (KParams::rb_*): the first block index past one residency round (step_kernel's issue priority)
// and the slice size of the fused rollout.
template <bool NOISE, bool DR, int PHYS, int SPEC>
static hipError_t occupancy_t(KParams& P) {
    int dev = 0, cus = 0, per_step = 0, per_roll = 0, per_collect = 0, per_croll_small = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_step, step_kernel<NOISE, DR, PHYS, SPEC>, STEP_BLOCK, 0);
    if (e == hipSuccess)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_roll, rollout_kernel<NOISE, DR, PHYS, SPEC>, STEP_BLOCK, 0);
    if constexpr (NOISE && SPEC == 1 && PHYS == PHYS_BULLET_T)
        if (e == hipSuccess)
            e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_collect, collect_kernel<NOISE, DR, PHYS, SPEC>,
                                                             STEP_BLOCK, 0);
    if constexpr (NOISE && SPEC == 1 && PHYS == PHYS_BULLET_T)
        if (e == hipSuccess)
            e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &per_croll_small, collect_rollout_kernel_small<NOISE, DR, PHYS, SPEC>, CROLL_SMALL_BLOCK, 0);
    if (e != hipSuccess) return e;
    P.rb_step = (uint32_t)(cus * (per_step > 0 ? per_step : 1));
    P.rb_roll = (uint32_t)(cus * (per_roll > 0 ? per_roll : 1));
    P.rb_collect = (uint32_t)(cus * (per_collect > 0 ? per_collect : 1));
    P.rb_croll_small = (uint32_t)(cus * (per_croll_small > 0 ? per_croll_small : 1));
    return hipSuccess;
}

template <bool NOISE, bool DR, int PHYS, int SPEC>
static hipError_t launch_step_t(const KParams& P, const StepIO& io, hipStream_t s, const PackIO& X = PackIO{}) {
    // small N (<= 32768 envs: at most one 64-env wave per two SIMDs with the helpers) runs 64 envs
    // per block, the other three waves computing the envs' potential resets meanwhile
    // (step_kernel_small); above that the helper waves would cost residency (65 536 envs: 15.5 ->
    // 24.7 us with 64-env blocks)
    if (P.N <= SMALL_N_MAX) {
        hipLaunchKernelGGL((step_kernel_small<NOISE, DR, PHYS, SPEC>), dim3((P.N + 63u) / 64u), dim3(256), 0, s, P, io, X);
        return hipGetLastError();
    }
    const dim3 grid((P.N + STEP_BLOCK - 1) / STEP_BLOCK), block(STEP_BLOCK);
    KParams Pl = P;
    Pl.late_block = P.rb_step;
    // the env state plus the step's I/O no longer fit the 256 MB Infinity Cache between env-steps
    // (P.nt_state, cf2_create): stream the state stores past it (nt), HBM-bound regime
    if (P.nt_state) {
        hipLaunchKernelGGL((step_kernel<NOISE, DR, PHYS, SPEC, 2>), grid, block, 0, s, Pl, io, X);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((step_kernel<NOISE, DR, PHYS, SPEC>), grid, block, 0, s, Pl, io, X);
    return hipGetLastError();
}
template <bool NOISE, bool DR, int PHYS, int SPEC>
static hipError_t launch_collect_t(const KParams& P, const StepIO& io, const PolicyIO& pio, hipStream_t s) {
    if constexpr (!NOISE || SPEC != 1 || PHYS != PHYS_BULLET_T) {
        return hipErrorNotSupported;
    } else {
        if (P.N <= SMALL_N_MAX) {     // small N: 64-env blocks with helper waves (as launch_step_t)
            hipLaunchKernelGGL((collect_kernel_small<NOISE, DR, PHYS, SPEC>), dim3((P.N + 63u) / 64u), dim3(256), 0, s,
                               P, io, pio);
            return hipGetLastError();
        }
        KParams Pl = P;
        Pl.late_block = P.rb_collect;
        hipLaunchKernelGGL((collect_kernel<NOISE, DR, PHYS, SPEC>), dim3((P.N + STEP_BLOCK - 1) / STEP_BLOCK),
                           dim3(STEP_BLOCK), 0, s, Pl, io, pio);
        return hipGetLastError();
    }
}
template <bool NOISE, bool DR, int PHYS, int SPEC>
static hipError_t launch_rollout_t(const KParams& P, const StepIO& io, uint32_t K, uint32_t act_stride, hipStream_t s) {
    // envs are processed in slices that fit one residency round (P.rb_roll blocks resident at
    // once): a slice's blocks run all K steps together, so no block waits K steps for a free slot.
    // Slices run one after the other on the stream.  Small N: 64 envs per block, the other waves
    // help with the resets (as launch_step_t).
    const uint32_t epb = P.N <= SMALL_N_MAX ? 64u : STEP_BLOCK;
    const uint32_t blocks = (P.N + epb - 1) / epb;
    const uint32_t round_blocks = P.rb_roll > 0 ? P.rb_roll : 1u;
    const uint32_t nslices = (blocks + round_blocks - 1) / round_blocks;
    const uint32_t per = (blocks + nslices - 1) / nslices;           // blocks per slice (balanced)
    constexpr int OD = NOISE ? 34 : 42;
    for (uint32_t b0 = 0; b0 < blocks; b0 += per) {
        const uint32_t nb = blocks - b0 < per ? blocks - b0 : per;
        const uint32_t e0 = b0 * epb;
        KParams Ps = P;
        Ps.N = (P.N - e0 < nb * epb) ? P.N - e0 : nb * epb;
        Ps.gid_off = P.gid_off + e0;
        // a slice sees its envs as 0..Ps.N-1: the state view starts at its first tile (e0 is a
        // multiple of 64), each output at its first row; the per-step slab stride
        // stays that of the whole population (rollout_kernel strides by its own Ps.N, so the
        // outputs of a sliced launch use an explicit stride below)
        StepIO ios = io;
        ios.sf = io.sf + (size_t)(e0 / 64u) * (NG * 256);
        ios.act = io.act + (size_t)e0 * 4;
        ios.obs = io.obs + (size_t)e0 * OD;
        ios.rew = io.rew + e0;
        ios.done = io.done + e0;
        if (io.trunc) ios.trunc = io.trunc + e0;
        if (io.cost) ios.cost = io.cost + e0;
        if (io.level) ios.level = io.level + e0;
        if (io.final_obs) ios.final_obs = io.final_obs + (size_t)e0 * OD;
        Ps.out_stride = P.N;
        if (epb == 64u)
            hipLaunchKernelGGL((rollout_kernel_small<NOISE, DR, PHYS, SPEC>), dim3(nb), dim3(256), 0, s, Ps, ios, K,
                               act_stride);
        else
            hipLaunchKernelGGL((rollout_kernel<NOISE, DR, PHYS, SPEC>), dim3(nb), dim3(STEP_BLOCK), 0, s, Ps, ios, K,
                               act_stride);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}
template <bool NOISE, bool DR, int PHYS, int SPEC>
static hipError_t launch_collect_rollout_t(const KParams& P, const StepIO& io, const PolicyIO& pio, uint32_t K,
                                           hipStream_t s) {
    if constexpr (!NOISE || SPEC != 1 || PHYS != PHYS_BULLET_T) {
        return hipErrorNotSupported;
    } else {
        constexpr uint32_t OD = 34;
        if (P.N > SMALL_N_MAX) {
            // large N: one collect_kernel launch per env-step.  A one-launch version (rollout_kernel's
            // env-step with the state in registers + this policy phase, 2 blocks per CU) was
            // bit-identical but slower at 262 144 envs, 65.0 against 60.3 us per env-step
            // (tools/variants/collect_rollout_large.hip.txt, profiles/r04_collect_ab.txt)
            for (uint32_t k = 0; k < K; ++k) {
                StepIO iok = io;
                iok.act = pio.act + (size_t)k * P.N * 4;
                iok.obs = io.obs + (size_t)k * P.N * OD;
                iok.rew = io.rew + (size_t)k * P.N;
                iok.done = io.done + (size_t)k * P.N;
                if (io.trunc) iok.trunc = io.trunc + (size_t)k * P.N;
                if (io.final_obs) iok.final_obs = io.final_obs + (size_t)k * P.N * OD;
                PolicyIO pk = pio;
                pk.counter = pio.counter + k;
                pk.act = pio.act + (size_t)(k + 1) * P.N * 4;
                pk.val = pio.val + (size_t)(k + 1) * P.N;
                pk.logp = pio.logp + (size_t)(k + 1) * P.N;
                const hipError_t e = launch_collect_t<NOISE, DR, PHYS, SPEC>(P, iok, pk, s);
                if (e != hipSuccess) return e;
            }
            return hipSuccess;
        }
        // small N: 128-env blocks of two helper-wave groups (collect_rollout_kernel_small), one per
        // CU, in slices of one residency round each (as launch_rollout_t): a slice's blocks run all
        // K steps together.  Every output slab keeps the whole population's stride.
        constexpr uint32_t epb = 128u;
        const uint32_t blocks = (P.N + epb - 1) / epb;
        const uint32_t round_blocks = P.rb_croll_small > 0 ? P.rb_croll_small : 1u;
        const uint32_t nslices = (blocks + round_blocks - 1) / round_blocks;
        const uint32_t per = (blocks + nslices - 1) / nslices;
        for (uint32_t b0 = 0; b0 < blocks; b0 += per) {
            const uint32_t nb = blocks - b0 < per ? blocks - b0 : per;
            const uint32_t e0 = b0 * epb;
            KParams Ps = P;
            Ps.N = (P.N - e0 < nb * epb) ? P.N - e0 : nb * epb;
            Ps.gid_off = P.gid_off + e0;
            Ps.out_stride = P.N;
            StepIO ios = io;
            ios.sf = io.sf + (size_t)(e0 / 64u) * (NG * 256);
            ios.obs = io.obs + (size_t)e0 * OD;
            ios.rew = io.rew + e0;
            ios.done = io.done + e0;
            if (io.trunc) ios.trunc = io.trunc + e0;
            if (io.final_obs) ios.final_obs = io.final_obs + (size_t)e0 * OD;
            PolicyIO ps = pio;
            ps.row_offset = pio.row_offset + e0;
            ps.act = pio.act + (size_t)e0 * 4;
            ps.val = pio.val + e0;
            ps.logp = pio.logp + e0;
            hipLaunchKernelGGL((collect_rollout_kernel_small<NOISE, DR, PHYS, SPEC>), dim3(nb), dim3(CROLL_SMALL_BLOCK), 0,
                               s, Ps, ios, ps, K);
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
}
template <bool NOISE, bool DR, int PHYS, int SPEC>
static hipError_t launch_reset_t(const KParams& P, float* sf, const uint8_t* mask, float* obs, hipStream_t s) {
    const dim3 grid((P.N + 255) / 256), block(256);
    hipLaunchKernelGGL((reset_kernel<NOISE, DR, PHYS, SPEC>), grid, block, 0, s, P, sf, mask, obs);
    return hipGetLastError();
}

// SPEC 1 when the config has the reference-default Bullet env-step shape (see shape_view), SPEC 2
// for the same shape flown in multi-drone formations
static inline bool spec_default_shape(const KParams& P) {
    return P.phys == PHYS_BULLET_T && P.agg == 2 && P.obs_rate == 2 && P.buf_size == 2 && P.use_latency &&
           P.use_motor_dyn;
}

#define CF2_DISPATCH(FN, ...)                                                                          \
    do {                                                                                               \
        const int key = (P.noise ? 4 : 0) | (P.dr ? 2 : 0) | (P.phys == PHYS_SIMPLE_T ? 1 : 0);           \
        if (spec_default_shape(P) && P.num_drones == 1) {                                              \
            switch (key) {                                                                             \
            case 0: return FN<false, false, PHYS_BULLET_T, 1>(__VA_ARGS__);                            \
            case 2: return FN<false, true, PHYS_BULLET_T, 1>(__VA_ARGS__);                             \
            case 4: return FN<true, false, PHYS_BULLET_T, 1>(__VA_ARGS__);                             \
            default: return FN<true, true, PHYS_BULLET_T, 1>(__VA_ARGS__);                             \
            }                                                                                          \
        }                                                                                              \
        if (spec_default_shape(P)) {                                                                   \
            switch (key) {                                                                             \
            case 0: return FN<false, false, PHYS_BULLET_T, 2>(__VA_ARGS__);                            \
            case 2: return FN<false, true, PHYS_BULLET_T, 2>(__VA_ARGS__);                             \
            case 4: return FN<true, false, PHYS_BULLET_T, 2>(__VA_ARGS__);                             \
            default: return FN<true, true, PHYS_BULLET_T, 2>(__VA_ARGS__);                             \
            }                                                                                          \
        }                                                                                              \
        switch (key) {                                                                                 \
        case 0: return FN<false, false, PHYS_BULLET_T, 0>(__VA_ARGS__);                                \
        case 1: return FN<false, false, PHYS_SIMPLE_T, 0>(__VA_ARGS__);                                \
        case 2: return FN<false, true, PHYS_BULLET_T, 0>(__VA_ARGS__);                                 \
        case 3: return FN<false, true, PHYS_SIMPLE_T, 0>(__VA_ARGS__);                                 \
        case 4: return FN<true, false, PHYS_BULLET_T, 0>(__VA_ARGS__);                                 \
        case 5: return FN<true, false, PHYS_SIMPLE_T, 0>(__VA_ARGS__);                                 \
        case 6: return FN<true, true, PHYS_BULLET_T, 0>(__VA_ARGS__);                                  \
        default: return FN<true, true, PHYS_SIMPLE_T, 0>(__VA_ARGS__);                                 \
        }                                                                                              \
    } while (0)

#ifdef CF2_TIMING
extern "C" int cf2_debug_timing_buffer(uint64_t* dev) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_cf2_timing), &dev, sizeof(dev));
}
#endif
hipError_t query_occupancy(KParams& P) { CF2_DISPATCH(occupancy_t, P); }
hipError_t launch_step(const KParams& P, const StepIO& io, hipStream_t s) { CF2_DISPATCH(launch_step_t, P, io, s); }
hipError_t launch_step_packed(const KParams& P, const StepIO& io, const PackIO& pio, hipStream_t s) {
    CF2_DISPATCH(launch_step_t, P, io, s, pio);
}
hipError_t launch_rollout(const KParams& P, const StepIO& io, uint32_t K, uint32_t act_stride, hipStream_t s) {
    CF2_DISPATCH(launch_rollout_t, P, io, K, act_stride, s);
}
hipError_t launch_collect(const KParams& P, const StepIO& io, const PolicyIO& pio, hipStream_t s) {
    CF2_DISPATCH(launch_collect_t, P, io, pio, s);
}
hipError_t launch_collect_rollout(const KParams& P, const StepIO& io, const PolicyIO& pio, uint32_t K, hipStream_t s) {
    CF2_DISPATCH(launch_collect_rollout_t, P, io, pio, K, s);
}
hipError_t launch_reset(const KParams& P, float* sf, const uint8_t* mask, float* obs, hipStream_t s) {
    CF2_DISPATCH(launch_reset_t, P, sf, mask, obs, s);
}
template <bool NOISE, bool DR, int PHYS>
static hipError_t launch_physics_t(const KParams& P, float* sf, const float* act, const float* dstb, float dt_override,
                                   hipStream_t s) {
    const dim3 grid((P.N + 255) / 256), block(256);
    hipLaunchKernelGGL((physics_kernel<NOISE, DR, PHYS>), grid, block, 0, s, P, sf, act, dstb, dt_override);
    return hipGetLastError();
}
hipError_t launch_physics(const KParams& P, float* sf, const float* act, const float* dstb, float dt_override,
                          hipStream_t s) {
    switch ((P.noise ? 4 : 0) | (P.dr ? 2 : 0) | (P.phys == PHYS_SIMPLE_T ? 1 : 0)) {
    case 0: return launch_physics_t<false, false, PHYS_BULLET_T>(P, sf, act, dstb, dt_override, s);
    case 1: return launch_physics_t<false, false, PHYS_SIMPLE_T>(P, sf, act, dstb, dt_override, s);
    case 2: return launch_physics_t<false, true, PHYS_BULLET_T>(P, sf, act, dstb, dt_override, s);
    case 3: return launch_physics_t<false, true, PHYS_SIMPLE_T>(P, sf, act, dstb, dt_override, s);
    case 4: return launch_physics_t<true, false, PHYS_BULLET_T>(P, sf, act, dstb, dt_override, s);
    case 5: return launch_physics_t<true, false, PHYS_SIMPLE_T>(P, sf, act, dstb, dt_override, s);
    case 6: return launch_physics_t<true, true, PHYS_BULLET_T>(P, sf, act, dstb, dt_override, s);
    default: return launch_physics_t<true, true, PHYS_SIMPLE_T>(P, sf, act, dstb, dt_override, s);
    }
}
hipError_t launch_state_convert(const KParams& P, float* sf, float* state_f, int32_t* state_i, int to_public,
                                hipStream_t s) {
    const dim3 grid((P.N + 255) / 256), block(256);
    hipLaunchKernelGGL(state_convert_kernel, grid, block, 0, s, P.N, sf, state_f, state_i, to_public, (int)P.noise);
    return hipGetLastError();
}
hipError_t launch_init(const KParams& P, float* sf, hipStream_t s) {
    const dim3 grid((P.N + 255) / 256), block(256);
    hipLaunchKernelGGL(init_kernel, grid, block, 0, s, P, sf);
    return hipGetLastError();
}
hipError_t launch_hj_sign_table(const float* V, uint32_t num_tables, uint8_t* bits, hipStream_t s) {
    const uint32_t total = num_tables * (uint32_t)HJ_TABLE;
    hipLaunchKernelGGL(hj_sign_table_kernel, dim3((total + 255) / 256), dim3(256), 0, s, V, total, bits);
    return hipGetLastError();
}

hipError_t launch_hj(const HjGrid& G, const double umax[3], const float* V, const float* states, uint32_t n,
                     float level, float* dstb, float* uopt, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const dim3 grid((n + 255) / 256), block(256);
    const double3 um = make_double3(umax[0], umax[1], umax[2]);
    hipLaunchKernelGGL(hj_kernel, grid, block, 0, s, G, um, V, states, n, level, dstb, uopt);
    return hipGetLastError();
}

}  // namespace cf2
