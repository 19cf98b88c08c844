// cf2sim_policy.h -- device-side pieces of the fused Gaussian MLP actor-critic forward (SURVEY
// section 8, row f3), shared by policy_kernel (cf2sim_policy.hip) and the fused env-step + policy
// kernel of the collect loop (collect_kernel, cf2sim_kernels.hip).  The formulation (transposed
// layers on the matrix cores, split-bf16 products, fragment packing) is described at the top of
// cf2sim_policy.hip.  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "cf2sim_rng.h"
#include "../../include/cf2sim.h"

namespace cf2 {

typedef float f4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf8v __attribute__((ext_vector_type(8)));

template <int D>
struct PolicyLayout {
    static constexpr int P_W1 = 0, P_B1 = P_W1 + D * 50, P_W2 = P_B1 + 50, P_B2 = P_W2 + 50 * 50, P_W3 = P_B2 + 50,
                         P_B3 = P_W3 + 50 * 4, P_LOGSTD = P_B3 + 4;
    static constexpr int V_W1 = P_LOGSTD + 4, V_B1 = V_W1 + D * 64, V_W2 = V_B1 + 64, V_B2 = V_W2 + 64 * 64,
                         V_W3 = V_B2 + 64, V_B3 = V_W3 + 64;
    static constexpr int O_MEAN = V_B3 + 1, O_SCALE = O_MEAN + D;     // observation standardisation
    static constexpr int TOTAL = O_SCALE + D;
};

// fp32 k-steps over a C-layout activation of 4 tiles with V valid neurons: step (t, i) holds
// neurons 16t + 4g + i (g = 0..3); steps with no valid neuron are skipped (pi: 50 -> 14, v: 16)
constexpr int ksteps(int V) {
    int n = 0;
    for (int t = 0; t < 4; ++t)
        for (int i = 0; i < 4; ++i) n += (16 * t + i < V) ? 1 : 0;
    return n;
}
constexpr int kstep_t(int V, int s) {
    for (int t = 0; t < 4; ++t)
        for (int i = 0; i < 4; ++i)
            if (16 * t + i < V && s-- == 0) return t;
    return -1;
}
constexpr int kstep_i(int V, int s) {
    for (int t = 0; t < 4; ++t)
        for (int i = 0; i < 4; ++i)
            if (16 * t + i < V && s-- == 0) return i;
    return -1;
}

// Neuron-level weights of the four GEMMs (0 for padding).  Layer 1 is the 128-wide [pi | v]
// layer (rows 0..49 pi, 64..127 v); layer 3 has rows 0..3 = mu, row 4 = v over the 128-wide
// [pi h2 | v h2] input (pi inputs 0..63, v inputs 64..127).
template <int D>
__device__ float w_l1(const float* __restrict__ W, int n, int in) {
    using L = PolicyLayout<D>;
    if (in >= D) return 0.0f;
    if (n < 64) return n < 50 ? W[L::P_W1 + in * 50 + n] : 0.0f;
    return W[L::V_W1 + in * 64 + (n - 64)];
}
template <int D>
__device__ float w_l2p(const float* __restrict__ W, int n, int in) {
    return (n < 50 && in < 50) ? W[PolicyLayout<D>::P_W2 + in * 50 + n] : 0.0f;
}
template <int D>
__device__ float w_l2v(const float* __restrict__ W, int n, int in) { return W[PolicyLayout<D>::V_W2 + in * 64 + n]; }
template <int D>
__device__ float w_l3(const float* __restrict__ W, int n, int in) {
    using L = PolicyLayout<D>;
    if (in < 64) return (n < 4 && in < 50) ? W[L::P_W3 + in * 4 + n] : 0.0f;
    return n == 4 ? W[L::V_W3 + in - 64] : 0.0f;
}

// Packed block layout (floats).  fp32 fragments: 64 floats (lane l: A[16nt + (l&15)][k slot l>>4]).
// bf16 fragments: 512 floats = hi[64 lanes][8 bf16] then lo[64 lanes][8 bf16] (lane l: k slots
// 8(l>>4) .. 8(l>>4)+7).  Layer 1 in bf16x3 mode: D/32 bf16 blocks + fp32 k-steps for the rest.
template <int D, int PREC>
struct Packed {
    static constexpr bool BF = PREC == CF2_POLICY_BF16X3;
    static constexpr int KB1 = BF ? D / 32 : 0;                          // bf16 k-blocks of layer 1
    static constexpr int K1R = 32 * KB1;                                 // first input past them
    static constexpr int R1 = D - K1R;                                   // layer-1 inputs left over
    // the left-over inputs (D = 34: 2) run as fp32 k-steps.  Measured against one slot-packed bf16
    // MFMA per n-tile for their three split products: 34.2 vs 35.0 us at 262 144 rows (the kernel
    // is bound by vector issue, not by the matrix pipe)
    static constexpr int KS1 = BF ? (R1 + 3) / 4 : (D + 3) / 4;             // fp32 k-steps of layer 1
    static constexpr int KSP = ksteps(50), KSV = ksteps(64);
    static constexpr int FB = 512, FF = 64;
    static constexpr int O_L1B = 0, O_L1F = O_L1B + KB1 * 8 * FB, O_L2P = O_L1F + KS1 * 8 * FF;
    static constexpr int N_L2 = BF ? 2 * 4 * FB : 0;
    static constexpr int O_L2V = O_L2P + (BF ? N_L2 : KSP * 4 * FF);
    static constexpr int O_L3 = O_L2V + (BF ? N_L2 : KSV * 4 * FF);
    // layer 3 (5 outputs) on bf16 k-blocks in bf16x3 mode.  On fp32 k-steps its inputs would need
    // no hi/lo split (-97 VALU per chunk), for 30 fp32 MFMAs instead of 12 bf16 ones: measured
    // 38.7 vs 34.1 us, so the matrix pipe is as close to the limit as the VALU
    static constexpr bool L3F = !BF;
    static constexpr int O_BIAS = O_L3 + (L3F ? (KSP + KSV) * FF : 4 * FB);
    static constexpr int B_L1 = 0, B_L2P = 128, B_L2V = 192, B_L3 = 256, NB = 272;   // neuron-ordered biases
    static constexpr int O_LOGSTD = O_BIAS + NB, O_MEAN = O_LOGSTD + 4, O_SCALE = O_MEAN + (D + 3) / 4 * 4;
    static constexpr int TOTAL = (O_SCALE + D + 3) / 4 * 4;
};

// bf16x3 mode packs the v network's layer-1 and layer-2 weights and biases multiplied by
// TANH_PRESCALE = -2 log2(e), so that its tanh needs no scaling (tanh_prescaled below)
constexpr float TANH_PRESCALE = -2.8853900817779268f;
template <int PREC>
__device__ __forceinline__ float v_prescale(bool v_pre_tanh) {
    return (PREC == CF2_POLICY_BF16X3 && v_pre_tanh) ? TANH_PRESCALE : 1.0f;
}

template <int D>
__device__ float bias_value(const float* __restrict__ W, int k) {
    using L = PolicyLayout<D>;
    if (k < 128) return k < 50 ? W[L::P_B1 + k] : (k < 64 ? 0.0f : W[L::V_B1 + k - 64]);
    if (k < 192) { const int n = k - 128; return n < 50 ? W[L::P_B2 + n] : 0.0f; }
    if (k < 256) return W[L::V_B2 + k - 192];
    const int n = k - 256;
    return n < 4 ? W[L::P_B3 + n] : (n == 4 ? W[L::V_B3] : 0.0f);
}

// bf16 k-block element: fragment (layer, kb, nt), lane l, slot j -> weight
template <int D>
__device__ float bf16_weight(const float* __restrict__ W, int layer, int kb, int nt, int l, int j) {
    const int n = 16 * nt + (l & 15), g = l >> 4;
    if (layer == 1) return w_l1<D>(W, n, 32 * kb + 8 * g + j);
    const int in = 16 * (2 * kb + (j >> 2)) + 4 * g + (j & 3);      // C-layout input, two tiles per block
    if (layer == 2) return w_l2p<D>(W, n, in);
    if (layer == 3) return w_l2v<D>(W, n, in);
    return w_l3<D>(W, n, in);                                          // kb 0,1: pi h2; 2,3: v h2 (+64)
}

__device__ __forceinline__ uint32_t bf16_bits(float x) {
    const __bf16 h = (__bf16)x;
    return (uint32_t)__builtin_bit_cast(uint16_t, h);
}

__device__ __forceinline__ f4v mfma4(float a, float b, f4v c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// split-bf16 product of one 32-k block: small terms first, then hi*hi
__device__ __forceinline__ f4v mfma3(const bf8v& ah, const bf8v& al, const bf8v& bh, const bf8v& bl, f4v c) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
}
// x -> (hi, lo) bf16 operands
typedef float f2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf2v __attribute__((ext_vector_type(2)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void split8(const float (&x)[8], bf8v& hi, bf8v& lo) {
    // two values per v_cvt_pk_bf16_f32: hi pair, its two fp32 values by shift / mask, the two
    // remainders, lo pair (6 VALU per pair; per-value conversions cost ~8)
    u4v h, o;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const f2v v = {x[2 * p], x[2 * p + 1]};
        const uint32_t hb = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf2v));
        const f2v r = {v.x - __uint_as_float(hb << 16), v.y - __uint_as_float(hb & 0xffff0000u)};
        h[p] = hb;
        o[p] = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, bf2v));
    }
    hi = __builtin_bit_cast(bf8v, h);
    lo = __builtin_bit_cast(bf8v, o);
}
// B operand of k-block (t0, t0 + 1) from two C-layout tiles
__device__ __forceinline__ void split_tiles(const f4v& a, const f4v& b, bf8v& hi, bf8v& lo) {
    const float x[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    split8(x, hi, lo);
}
__device__ __forceinline__ void ld_frag(const float* sw, int off, int l, bf8v& hi, bf8v& lo) {
    const float4 h = *reinterpret_cast<const float4*>(sw + off + 4 * l);
    const float4 o = *reinterpret_cast<const float4*>(sw + off + 256 + 4 * l);
    hi = __builtin_bit_cast(bf8v, h);
    lo = __builtin_bit_cast(bf8v, o);
}

// tanh(x) = sign(x) (1 - 2 / (exp(2|x|) + 1)) on v_exp_f32 / v_rcp_f32 (abs error < 2e-7)
__device__ __forceinline__ float tanh_fast(float x) {
    const float e = __builtin_amdgcn_exp2f(2.8853900817779268f * fabsf(x));   // exp(2|x|)
    return __builtin_copysignf(1.0f - 2.0f * __builtin_amdgcn_rcpf(e + 1.0f), x);
}
// tanh(z) from y = -2 log2(e) z (the v network's layer-1 and layer-2 weights and biases are packed
// pre-multiplied by TANH_PRESCALE in bf16x3 mode): 2 / (1 + 2^y) - 1, 4 VALU against 6.  Saturates
// correctly (2^y -> inf: -1; 2^y -> 0: 1); absolute error ~2e-7 near 0, as tanh_fast.
__device__ __forceinline__ float tanh_prescaled(float y) {
    return fmaf(2.0f, __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(y)), -1.0f);
}
// ReLU as an integer max on the bits (negative floats, -0 included, are negative integers): one
// v_max_i32; fmaxf(x, 0) on an MFMA result costs two v_max_f32 (IEEE-mode NaN quieting first)
__device__ __forceinline__ float relu(float x) {
    return __int_as_float(__builtin_elementwise_max(__float_as_int(x), 0));
}
template <int PREC>
__device__ __forceinline__ float tanh_act(float x) {
    if constexpr (PREC == CF2_POLICY_BF16X3) return tanh_prescaled(x);
    else return tanh_fast(x);
}

enum : uint32_t { TAG_POLICY = 3 };
// One row tile per chunk, 8-wave blocks, 4 waves per SIMD: bf16x3 41.5 -> 38.6 us and fp32
// 81.4 -> 76.5 us at 262 144 rows against 2 row tiles per chunk in 4-wave blocks at 2 waves per
// SIMD (each fragment read then feeds one MFMA instead of two, but twice as many waves hide the
// LDS and MFMA latencies; 3 waves/SIMD in 6-wave blocks: 50.1 us; 16-wave blocks: 40.2 us)
constexpr int RT = 1;             // row tiles (16 rows each) per wave chunk: each fragment read feeds RT MFMAs
constexpr int CHUNK = 16 * RT;
constexpr int PB = 512, PW = PB / 64;   // threads per block (one staged copy of the fragments per block)
constexpr int POLICY_WAVES = 4;   // waves per SIMD the register budget is sized for

// The observations of one chunk, raw fp32: per row tile the bf16 k-blocks' 8 consecutive inputs
// of this lane's group (x8) and the fp32 k-steps' single inputs (x1).  Loads are unconditional
// (indices clamped into the buffer): a row past n is never written out and an input index past
// D meets a zero weight; branch-free loads keep the waitcnt counting exact, so the prefetch of
// the next chunk stays in flight under this chunk's MFMAs.
template <int D, int PREC, int R = RT>
struct ObsRegs {
    using P = Packed<D, PREC>;
    float x8[R][P::KB1 > 0 ? P::KB1 : 1][8];
    float x1[R][P::KS1 > 0 ? P::KS1 : 1];
};
template <int D, int PREC>
__device__ __forceinline__ void load_obs(const float* __restrict__ obs, uint32_t n, uint32_t r0, int l,
                                         ObsRegs<D, PREC>& X) {
    using P = Packed<D, PREC>;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const uint32_t row = __builtin_elementwise_min(r0 + 16 * rt + (uint32_t)(l & 15), n - 1u);
        const float* src = obs + (size_t)row * D;
#pragma unroll
        for (int kb = 0; kb < P::KB1; ++kb)
#pragma unroll
            for (int q = 0; q < 4; ++q) {     // rows are 8-B aligned (D even): 4 x float2
                const float2 v = *reinterpret_cast<const float2*>(src + 32 * kb + 8 * (l >> 4) + 2 * q);
                X.x8[rt][kb][2 * q] = v.x;
                X.x8[rt][kb][2 * q + 1] = v.y;
            }
#pragma unroll
        for (int ks = 0; ks < P::KS1; ++ks)
            X.x1[rt][ks] = src[__builtin_elementwise_min(P::K1R + 4 * ks + (l >> 4), D - 1)];
    }
}

// ---- the forward of one chunk, shared by policy_kernel and the fused env + policy kernel
// (collect_kernel in cf2sim_kernels.hip).  Pointers: sw = the fragments (LDS; the layer-1 and
// layer-2 offsets of Packed), sb = the packed block's tail from O_BIAS on (biases, log_std,
// standardisation constants; LDS), l3 = the layer-3 fragments (LDS in policy_kernel; global
// memory in the fused kernel, whose LDS holds everything but them).
template <int D, int PREC>
struct PolicyLane {     // per-lane constants, hoisted out of the chunk loop
    using P = Packed<D, PREC>;
    float ls[4], sd[4];
    float mean1[P::KS1 > 0 ? P::KS1 : 1], scale1[P::KS1 > 0 ? P::KS1 : 1];
};
template <int D, int PREC>
__device__ __forceinline__ void policy_lane_init(const float* sb, int g, PolicyLane<D, PREC>& C) {
    using P = Packed<D, PREC>;
    constexpr int T_LOGSTD = P::O_LOGSTD - P::O_BIAS, T_MEAN = P::O_MEAN - P::O_BIAS, T_SCALE = P::O_SCALE - P::O_BIAS;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        C.ls[k] = sb[T_LOGSTD + k];
        C.sd[k] = __builtin_amdgcn_exp2f(1.4426950408889634f * C.ls[k]);
    }
#pragma unroll
    for (int ks = 0; ks < P::KS1; ++ks) {
        const int k = __builtin_elementwise_min(P::K1R + 4 * ks + g, D - 1);
        C.mean1[ks] = sb[T_MEAN + k];
        C.scale1[ks] = sb[T_SCALE + k];
    }
}

// observation standardisation (obs - mean) * scale, per input index of this lane; the k-block
// constants are re-read from LDS per chunk (16 fewer live VGPRs than holding them)
template <int D, int PREC, int R = RT>
__device__ __forceinline__ void policy_standardize(const float* sb, int g, const PolicyLane<D, PREC>& C,
                                                   ObsRegs<D, PREC, R>& Xc) {
    using P = Packed<D, PREC>;
    constexpr int T_MEAN = P::O_MEAN - P::O_BIAS, T_SCALE = P::O_SCALE - P::O_BIAS;
    float mean8[P::KB1 > 0 ? P::KB1 : 1][8], scale8[P::KB1 > 0 ? P::KB1 : 1][8];
#pragma unroll
    for (int kb = 0; kb < P::KB1; ++kb)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const float4 m = *reinterpret_cast<const float4*>(&sb[T_MEAN + 32 * kb + 8 * g + 4 * q]);
            const float4 sc = *reinterpret_cast<const float4*>(&sb[T_SCALE + 32 * kb + 8 * g + 4 * q]);
            mean8[kb][4 * q] = m.x; mean8[kb][4 * q + 1] = m.y; mean8[kb][4 * q + 2] = m.z; mean8[kb][4 * q + 3] = m.w;
            scale8[kb][4 * q] = sc.x; scale8[kb][4 * q + 1] = sc.y; scale8[kb][4 * q + 2] = sc.z; scale8[kb][4 * q + 3] = sc.w;
        }
#pragma unroll
    for (int rt = 0; rt < R; ++rt) {
#pragma unroll
        for (int kb = 0; kb < P::KB1; ++kb)
#pragma unroll
            for (int j = 0; j < 8; ++j) Xc.x8[rt][kb][j] = (Xc.x8[rt][kb][j] - mean8[kb][j]) * scale8[kb][j];
#pragma unroll
        for (int ks = 0; ks < P::KS1; ++ks) Xc.x1[rt][ks] = (Xc.x1[rt][ks] - C.mean1[ks]) * C.scale1[ks];
    }
}

// layers 1-3 on standardised inputs.  MODE 0: both networks (o: lanes 0..15 mu[0..3] of row
// l & 15, lanes 16..31 v in register 0); MODE 1: the v network only.
template <int D, int PREC, int MODE, int R = RT>
__device__ __forceinline__ void policy_layers(const float* sw, const float* sb, const float* l3, int l,
                                              const ObsRegs<D, PREC, R>& Xc, f4v (&o)[R]) {
    constexpr int RT = R;      // row tiles of this call (each fragment read feeds R MFMAs)
    using P = Packed<D, PREC>;
    constexpr bool PI = MODE == 0, BF = P::BF;
    constexpr int T_BIAS = 0;
    const int g = l >> 4;
    // ---- layer 1: [pi | v] 128 neurons (8 n-tiles); MODE 1 runs only the v half
    constexpr int NT0 = PI ? 0 : 4;
    f4v h1[8][RT];
#pragma unroll
    for (int nt = NT0; nt < 8; ++nt) {
        const f4v b = *reinterpret_cast<const f4v*>(&sb[T_BIAS + P::B_L1 + 16 * nt + 4 * g]);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) h1[nt][rt] = b;
    }
#pragma unroll
    for (int kb = 0; kb < P::KB1; ++kb) {
        bf8v bh[RT], bl[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) split8(Xc.x8[rt][kb], bh[rt], bl[rt]);
#pragma unroll
        for (int nt = NT0; nt < 8; ++nt) {
            bf8v ah, al;
            ld_frag(sw, P::O_L1B + (kb * 8 + nt) * P::FB, l, ah, al);
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) h1[nt][rt] = mfma3(ah, al, bh[rt], bl[rt], h1[nt][rt]);
        }
    }
#pragma unroll
    for (int ks = 0; ks < P::KS1; ++ks)
#pragma unroll
        for (int nt = NT0; nt < 8; ++nt) {
            const float a = sw[P::O_L1F + (ks * 8 + nt) * P::FF + l];
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) h1[nt][rt] = mfma4(a, Xc.x1[rt][ks], h1[nt][rt]);
        }
#pragma unroll
    for (int nt = NT0; nt < 8; ++nt)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int i = 0; i < 4; ++i) h1[nt][rt][i] = nt < 4 ? relu(h1[nt][rt][i]) : tanh_act<PREC>(h1[nt][rt][i]);
    // ---- layer 2: pi 50 -> 50 (ReLU), v 64 -> 64 (tanh); inputs straight from the layer-1 accumulators
    f4v h2p[4][RT], h2v[4][RT];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        const f4v bp = *reinterpret_cast<const f4v*>(&sb[T_BIAS + P::B_L2P + 16 * nt + 4 * g]);
        const f4v bv = *reinterpret_cast<const f4v*>(&sb[T_BIAS + P::B_L2V + 16 * nt + 4 * g]);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) { h2p[nt][rt] = bp; h2v[nt][rt] = bv; }
    }
#pragma unroll
    for (int half = PI ? 0 : 1; half < 2; ++half) {      // 0: pi, 1: v
        f4v(&acc)[4][RT] = half ? h2v : h2p;
        const int O = half ? P::O_L2V : P::O_L2P, T0 = half ? 4 : 0;
        if constexpr (BF) {
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
                bf8v bh[RT], bl[RT];
#pragma unroll
                for (int rt = 0; rt < RT; ++rt)
                    split_tiles(h1[T0 + 2 * kb][rt], h1[T0 + 2 * kb + 1][rt], bh[rt], bl[rt]);
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) {
                    bf8v ah, al;
                    ld_frag(sw, O + (kb * 4 + nt) * P::FB, l, ah, al);
#pragma unroll
                    for (int rt = 0; rt < RT; ++rt) acc[nt][rt] = mfma3(ah, al, bh[rt], bl[rt], acc[nt][rt]);
                }
            }
        } else {
            constexpr int V0 = 50, V1 = 64;
#pragma unroll
            for (int ks = 0; ks < (half ? P::KSV : P::KSP); ++ks) {
                const int t = half ? kstep_t(V1, ks) : kstep_t(V0, ks), i = half ? kstep_i(V1, ks) : kstep_i(V0, ks);
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) {
                    const float a = sw[O + (ks * 4 + nt) * P::FF + l];
#pragma unroll
                    for (int rt = 0; rt < RT; ++rt) acc[nt][rt] = mfma4(a, h1[T0 + t][rt][i], acc[nt][rt]);
                }
            }
        }
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (PI) h2p[nt][rt][i] = relu(h2p[nt][rt][i]);
                h2v[nt][rt][i] = tanh_act<PREC>(h2v[nt][rt][i]);
            }
    // ---- layer 3: one n-tile, rows 0..3 = mu, row 4 = v (fragments at l3)
    {
        const f4v b = *reinterpret_cast<const f4v*>(&sb[T_BIAS + P::B_L3 + 4 * g]);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) o[rt] = b;
    }
#pragma unroll
    for (int half = PI ? 0 : 1; half < 2; ++half) {
        f4v(&h)[4][RT] = half ? h2v : h2p;
        if constexpr (!P::L3F) {
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
                bf8v ah, al;
                ld_frag(l3, (2 * half + kb) * P::FB, l, ah, al);
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) {
                    bf8v bh, bl;
                    split_tiles(h[2 * kb][rt], h[2 * kb + 1][rt], bh, bl);
                    o[rt] = mfma3(ah, al, bh, bl, o[rt]);
                }
            }
        } else {
#pragma unroll
            for (int ks = 0; ks < (half ? P::KSV : P::KSP); ++ks) {
                const int t = half ? kstep_t(64, ks) : kstep_t(50, ks), i = half ? kstep_i(64, ks) : kstep_i(50, ks);
                const float a = l3[((half ? P::KSP : 0) + ks) * P::FF + l];
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) o[rt] = mfma4(a, h[t][rt][i], o[rt]);
            }
        }
    }
}

// Outputs of one row from the layer-3 tile (lanes 0..15 hold mu[0..3] of row 16 rt + l, lanes
// 16..31 hold v in register 0): the value, and in MODE 0 the Gaussian sample a = mu + std * eps
// and its log-probability (core.py:253-291), eps given (lanes 0..15)
template <int D, int PREC, int MODE>
__device__ __forceinline__ void policy_emit_eps(const f4v& o, uint32_t row, int g, const PolicyLane<D, PREC>& C,
                                                const float (&eps)[4], int sample, float* __restrict__ act,
                                                float* __restrict__ val, float* __restrict__ logp,
                                                const uint8_t* __restrict__ mask) {
    constexpr bool PI = MODE == 0;
    if (g == 1 && (MODE == 0 || mask[row])) val[row] = o[0];
    if (PI && g == 0) {
        float lp = 0.0f;
        float4 a;
        float* ap = &a.x;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            ap[k] = o[k] + C.sd[k] * eps[k];
            lp += -0.5f * eps[k] * eps[k] - C.ls[k] - 0.91893853320467274f;    // 0.5 log(2 pi)
        }
        reinterpret_cast<float4*>(act)[row] = a;
        if (logp) logp[row] = sample ? lp : 1.0f;
    }
}
// the sampling noise of one row: Philox(seed, counter, row_offset + row), two Box-Muller pairs
__device__ __forceinline__ void policy_noise(uint32_t key0, uint32_t key1, uint32_t counter, uint32_t prow,
                                             float (&eps)[4]) {
    const Keys K = make_keys(key0, key1);
    const U4 u = philox(K, 0u, counter, prow, TAG_POLICY);
    box_muller(u.x, u.y, eps[0], eps[1]);
    box_muller(u.z, u.w, eps[2], eps[3]);
}
template <int D, int PREC, int MODE>
__device__ __forceinline__ void policy_emit(const f4v& o, uint32_t row, int g, const PolicyLane<D, PREC>& C,
                                            uint32_t key0, uint32_t key1, uint32_t counter, uint32_t row_offset,
                                            int sample, float* __restrict__ act, float* __restrict__ val,
                                            float* __restrict__ logp, const uint8_t* __restrict__ mask) {
    float eps[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (MODE == 0 && g == 0 && sample) policy_noise(key0, key1, counter, row_offset + row, eps);
    policy_emit_eps<D, PREC, MODE>(o, row, g, C, eps, sample, act, val, logp, mask);
}

}  // namespace cf2
