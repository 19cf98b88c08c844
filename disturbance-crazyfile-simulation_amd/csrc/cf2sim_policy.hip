// cf2sim_policy.hip -- fused Gaussian MLP actor-critic forward for the batched rollout caller
// (SURVEY section 8, row f3).
//
// Restates, for a whole batch in one launch, ActorCritic.step of the reference
// (phoenix_drone_simulation/algs/core.py:371-395) with its PPO networks (algs/ppo/defaults.py:8-13):
//   pi: obs -> Linear(50) -> ReLU -> Linear(50) -> ReLU -> Linear(4) -> mu;  a = mu + exp(log_std) * eps
//       logp = Normal(mu, std).log_prob(a).sum(-1)                           (core.py:228-291)
//   v:  obs -> Linear(64) -> tanh -> Linear(64) -> tanh -> Linear(1)      (MLPCritic)
// As torch runs it, each layer is a separate GEMM plus an activation kernel, with 50- and 64-wide
// activations round-tripping through HBM (~0.6 ms per step at 262k rows).  Here the whole network
// runs on the matrix cores in one launch, fp32 activations and fp32 accumulation, in one of two
// product precisions (cf2_policy_precision in include/cf2sim.h):
//   CF2_POLICY_F32     v_mfma_f32_16x16x4_f32: exact fp32 (the result of an fmaf chain over k);
//   CF2_POLICY_BF16X3  v_mfma_f32_16x16x32_bf16 on split operands, x = hi + lo (two bf16 words),
//                      x*w ~ hi_x*hi_w + hi_x*lo_w + lo_x*hi_w: 16 significant bits per operand,
//                      <= ~3 * 2^-18 relative error per product (1.1e-5, typically a few 1e-6),
//                      at 3 bf16 MFMAs per 32-k block = 16/3 the fp32 rate.
//
// Transposed formulation: every layer computes out^T[neuron][row] = W[neuron][k] * in^T[k][row],
// weights as the A operand (16 neurons x k), activations as the B operand (k x 16 batch rows).
// The accumulator of an n-tile t holds, in lane l and register i, neuron 16t + 4(l>>4) + i of
// batch row l & 15.  Read as a B operand, that is a k-step whose k slot of lane group g = l >> 4
// is neuron 16t + 4g + i (fp32: one register per k-step of 4; bf16: two tiles' 8 registers per
// k-block of 32, slot (g, j) = neuron 16 t_{j/4} + 4g + (j % 4)).  The next layer's weights are
// packed in that permuted k order (cf2_policy_pack), so activations go from layer to layer in
// registers, with no LDS round trip and no cross-lane move.  Biases initialise the accumulators.
//
// Work split: persistent blocks of 8 waves, 2 per CU (4 waves per SIMD); each wave runs chunks of
// CF2_POLICY_RT row tiles of 16 rows and prefetches the next chunk's observations while the
// current one runs.  The packed block (A-operand fragments, lane-ordered:
// conflict-free ds_read_b32 / ds_read_b128) is staged into LDS once per block.
//
// Flat weight block (cf2_policy_weights_count floats; input-major so output neurons are contiguous):
//   pi: W1[D][50] b1[50] W2[50][50] b2[50] W3[50][4] b3[4] log_std[4]
//   v:  W1[D][64] b1[64] W2[64][64] b2[64] W3[64]    b3[1]
//   obs standardisation (core.py:383-388, OnlineMeanStd): mean[D], scale[D] = 1 / (std + 1e-5);
//   both networks see (obs - mean) * scale (identity: mean 0, scale 1)
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

#ifndef CF2_POLICY_L3F32
#define CF2_POLICY_L3F32 0
#endif
#ifndef CF2_POLICY_SLOT1
#define CF2_POLICY_SLOT1 0     // measured 35.0 vs 34.2 us at 262 144 rows: the kernel is VALU-, not MFMA-bound
#endif
// Packed block layout (floats).  fp32 fragments: 64 floats (lane l: A[16nt + (l&15)][k slot l>>4]).
// bf16 fragments: 512 floats = hi[64 lanes][8 bf16] then lo[64 lanes][8 bf16] (lane l: k slots
// 8(l>>4) .. 8(l>>4)+7).  Layer 1 in bf16x3 mode: D/32 bf16 blocks + fp32 k-steps for the rest.
template <int D, int PREC>
struct Packed {
    static constexpr bool BF = PREC == CF2_POLICY_BF16X3;
    static constexpr int KB1 = BF ? D / 32 : 0;                          // bf16 k-blocks of layer 1
    static constexpr int K1R = 32 * KB1;                                 // first input past them
    static constexpr int R1 = D - K1R;                                   // layer-1 inputs left over
    // bf16x3 with <= 2 left-over inputs (D = 34): their three split products hi*hi, lo_x*hi_w,
    // hi_x*lo_w share ONE bf16 MFMA per n-tile (k slots 0..3 R1-1 of lane group 0; a hi-only
    // fragment, FS floats) instead of fp32 k-steps (16 against 32 cycles per n-tile)
    static constexpr bool SL = BF && R1 > 0 && 3 * R1 <= 8 && CF2_POLICY_SLOT1;
    static constexpr int KS1 = SL ? 0 : (BF ? (R1 + 3) / 4 : (D + 3) / 4);   // fp32 k-steps of layer 1
    static constexpr int KSP = ksteps(50), KSV = ksteps(64);
    static constexpr int FB = 512, FF = 64, FS = 256;
    static constexpr int O_L1B = 0, O_L1F = O_L1B + KB1 * 8 * FB, O_L2P = O_L1F + KS1 * 8 * FF + (SL ? 8 * FS : 0);
    static constexpr int N_L2 = BF ? 2 * 4 * FB : 0;
    static constexpr int O_L2V = O_L2P + (BF ? N_L2 : KSP * 4 * FF);
    static constexpr int O_L3 = O_L2V + (BF ? N_L2 : KSV * 4 * FF);
    // layer 3 (5 outputs) on fp32 k-steps also in bf16x3 mode (CF2_POLICY_L3F32): its inputs need
    // no hi/lo split then (-97 VALU per chunk), for 30 fp32 MFMAs instead of 12 bf16 ones; measured
    // 38.7 vs 34.1 us, so the matrix pipe is as close to the limit as the VALU
    static constexpr bool L3F = !BF || CF2_POLICY_L3F32;
    static constexpr int O_BIAS = O_L3 + (L3F ? (KSP + KSV) * FF : 4 * FB);
    static constexpr int B_L1 = 0, B_L2P = 128, B_L2V = 192, B_L3 = 256, NB = 272;   // neuron-ordered biases
    static constexpr int O_LOGSTD = O_BIAS + NB, O_MEAN = O_LOGSTD + 4, O_SCALE = O_MEAN + (D + 3) / 4 * 4;
    static constexpr int TOTAL = (O_SCALE + D + 3) / 4 * 4;
};

// bf16x3 mode packs the v network's layer-1 and layer-2 weights and biases multiplied by
// TANH_PRESCALE = -2 log2(e), so that its tanh needs no scaling (tanh_prescaled below)
#ifndef CF2_POLICY_TANH_PRESCALE
#define CF2_POLICY_TANH_PRESCALE 1
#endif
constexpr float TANH_PRESCALE = -2.8853900817779268f;
template <int PREC>
__device__ __forceinline__ float v_prescale(bool v_pre_tanh) {
    return (PREC == CF2_POLICY_BF16X3 && CF2_POLICY_TANH_PRESCALE && v_pre_tanh) ? TANH_PRESCALE : 1.0f;
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

// one packed word per thread
template <int D, int PREC>
__global__ void __launch_bounds__(256) pack_kernel(const float* __restrict__ W, float* __restrict__ out) {
    using P = Packed<D, PREC>;
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= P::TOTAL) return;
    float v = 0.0f;
    auto bfword = [&](int layer, int rel, int nblk) -> float {
        // rel: offset inside this layer's bf16 fragments; nblk: n-tiles per k-block
        const int f = rel / P::FB, w = rel % P::FB, half = w / 256, lw = w % 256, l = lw / 4, pr = lw % 4;
        const int kb = f / nblk, nt = f % nblk;
        uint32_t bits = 0;
        const bool vt = layer == 3 || (layer == 1 && nt >= 4);     // v neurons before a tanh
        for (int e = 0; e < 2; ++e) {
            const float x = bf16_weight<D>(W, layer, kb, nt, l, 2 * pr + e) * v_prescale<PREC>(vt);
            const float hi = (float)(__bf16)x;
            bits |= (half ? bf16_bits(x - hi) : bf16_bits(x)) << (16 * e);
        }
        return __uint_as_float(bits);
    };
    if (k < P::O_L1F) {
        v = bfword(1, k - P::O_L1B, 8);
    } else if (k < P::O_L2P && P::SL) {
        // slot s of lane group 0: s < R1 hi(w), s < 2 R1 hi(w) (times lo(x)), s < 3 R1 lo(w)
        const int r = k - P::O_L1F, nt = r / P::FS, w = r % P::FS, l = w / 4, pr = w % 4;
        uint32_t bits = 0;
        for (int e = 0; e < 2; ++e) {
            const int sl = 2 * pr + e;
            if ((l >> 4) != 0 || sl >= 3 * P::R1) continue;
            const float x = w_l1<D>(W, 16 * nt + (l & 15), P::K1R + sl % P::R1) * v_prescale<PREC>(nt >= 4);
            const float hi = (float)(__bf16)x;
            bits |= (sl < 2 * P::R1 ? bf16_bits(x) : bf16_bits(x - hi)) << (16 * e);
        }
        v = __uint_as_float(bits);
    } else if (k < P::O_L2P) {
        const int r = k - P::O_L1F, f = r / 64, l = r % 64, ks = f / 8, nt = f % 8;
        v = w_l1<D>(W, 16 * nt + (l & 15), P::K1R + 4 * ks + (l >> 4)) * v_prescale<PREC>(nt >= 4);
    } else if (k < P::O_L2V) {
        const int r = k - P::O_L2P;
        if (P::BF) {
            v = bfword(2, r, 4);
        } else {
            const int f = r / 64, l = r % 64, ks = f / 4, nt = f % 4;
            v = w_l2p<D>(W, 16 * nt + (l & 15), 16 * kstep_t(50, ks) + 4 * (l >> 4) + kstep_i(50, ks));
        }
    } else if (k < P::O_L3) {
        const int r = k - P::O_L2V;
        if (P::BF) {
            v = bfword(3, r, 4);
        } else {
            const int f = r / 64, l = r % 64, ks = f / 4, nt = f % 4;
            v = w_l2v<D>(W, 16 * nt + (l & 15), 16 * kstep_t(64, ks) + 4 * (l >> 4) + kstep_i(64, ks));
        }
    } else if (k < P::O_BIAS) {
        const int r = k - P::O_L3;
        if (!P::L3F) {
            v = bfword(4, r, 1);
        } else {
            const int ks = r / 64, l = r % 64, n = l & 15, g = l >> 4;
            v = ks < P::KSP ? w_l3<D>(W, n, 16 * kstep_t(50, ks) + 4 * g + kstep_i(50, ks))
                            : w_l3<D>(W, n, 64 + 16 * kstep_t(64, ks - P::KSP) + 4 * g + kstep_i(64, ks - P::KSP));
        }
    } else if (k < P::O_LOGSTD) {
        const int b = k - P::O_BIAS;
        v = bias_value<D>(W, b) * v_prescale<PREC>((b >= 64 && b < 128) || (b >= P::B_L2V && b < P::B_L3));
    } else if (k < P::O_MEAN) {
        v = W[PolicyLayout<D>::P_LOGSTD + (k - P::O_LOGSTD)];
    } else if (k < P::O_SCALE) {
        v = k - P::O_MEAN < D ? W[PolicyLayout<D>::O_MEAN + (k - P::O_MEAN)] : 0.0f;     // 16-B aligned rows
    } else if (k < P::O_SCALE + D) {
        v = W[PolicyLayout<D>::O_SCALE + (k - P::O_SCALE)];
    }
    out[k] = v;
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
#ifndef CF2_POLICY_PAIRCVT
#define CF2_POLICY_PAIRCVT 1
#endif
typedef float f2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf2v __attribute__((ext_vector_type(2)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void split8(const float (&x)[8], bf8v& hi, bf8v& lo) {
#if CF2_POLICY_PAIRCVT
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
#else
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        hi[j] = (__bf16)x[j];
        lo[j] = (__bf16)(x[j] - (float)hi[j]);
    }
#endif
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
    if constexpr (PREC == CF2_POLICY_BF16X3 && CF2_POLICY_TANH_PRESCALE) return tanh_prescaled(x);
    else return tanh_fast(x);
}

enum : uint32_t { TAG_POLICY = 3 };
// One row tile per chunk, 8-wave blocks, 4 waves per SIMD: bf16x3 41.5 -> 38.6 us and fp32
// 81.4 -> 76.5 us at 262 144 rows against 2 row tiles per chunk in 4-wave blocks at 2 waves per
// SIMD (each fragment read then feeds one MFMA instead of two, but twice as many waves hide the
// LDS and MFMA latencies; 3 waves/SIMD in 6-wave blocks: 50.1 us; 16-wave blocks: 40.2 us)
#ifndef CF2_POLICY_RT
#define CF2_POLICY_RT 1          // row tiles (16 rows each) per wave chunk: each fragment read feeds RT MFMAs
#endif
#ifndef CF2_POLICY_BLOCK
#define CF2_POLICY_BLOCK 512     // threads per block (one staged copy of the fragments per block)
#endif
#ifndef CF2_POLICY_WAVES
#define CF2_POLICY_WAVES 4       // waves per SIMD the register budget is sized for
#endif
constexpr int RT = CF2_POLICY_RT;
constexpr int CHUNK = 16 * RT;
constexpr int PB = CF2_POLICY_BLOCK, PW = PB / 64;

// The observations of one chunk, raw fp32: per row tile the bf16 k-blocks' 8 consecutive inputs
// of this lane's group (x8) and the fp32 k-steps' single inputs (x1).  Loads are unconditional
// (indices clamped into the buffer): a row past n is never written out and an input index past
// D meets a zero weight; branch-free loads keep the waitcnt counting exact, so the prefetch of
// the next chunk stays in flight under this chunk's MFMAs.
template <int D, int PREC>
struct ObsRegs {
    using P = Packed<D, PREC>;
    float x8[RT][P::KB1 > 0 ? P::KB1 : 1][8];
    float x1[RT][P::KS1 > 0 ? P::KS1 : 1];
    float xr[RT][P::SL ? P::R1 : 1];
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
        if constexpr (P::SL)
#pragma unroll
            for (int r = 0; r < P::R1; ++r) X.xr[rt][r] = src[P::K1R + r];
    }
}

// mode: 0 = policy (mu, sample, logp) + value of every row; 1 = value only, rows with mask[r] != 0
template <int D, int PREC, int MODE>
__global__ void __launch_bounds__(PB, CF2_POLICY_WAVES) policy_kernel(const float* __restrict__ Wp, uint32_t n,
                                                                      const float* __restrict__ obs, uint32_t key0,
                                                                      uint32_t key1, uint32_t counter,
                                                                      uint32_t row_offset, int sample,
                                                                      float* __restrict__ act, float* __restrict__ val,
                                                                      float* __restrict__ logp,
                                                                      const uint8_t* __restrict__ mask) {
    using P = Packed<D, PREC>;
    constexpr bool PI = MODE == 0, BF = P::BF;
    __shared__ __align__(16) float s_w[P::TOTAL];
    const uint32_t nchunks = (n + CHUNK - 1) / CHUNK;
    const uint32_t wave = blockIdx.x * PW + (threadIdx.x >> 6), nwaves = gridDim.x * PW;
    if (MODE == 1) {
        // value-only pass (time-out bootstraps, usually no row marked): a block none of whose
        // chunks has a marked row exits before staging the weights
        // The block's chunks are runs of PW consecutive chunks, one run every nwaves chunks; the
        // block's m-th chunk is (m / PW) * nwaves + blockIdx.x * PW + m % PW. Each thread checks
        // whole chunks (CHUNK flag bytes, independent loads), so the scan is a few load latencies
        // rather than one per chunk of each wave.
        int any = 0;
        const uint32_t per_block = ((nchunks + nwaves - 1) / nwaves) * PW;
        for (uint32_t m = threadIdx.x; m < per_block; m += PB) {
            const uint32_t c = (m / PW) * nwaves + blockIdx.x * PW + m % PW;
            if (c >= nchunks) continue;
#pragma unroll
            for (int j = 0; j < CHUNK; ++j) {
                const uint32_t rr = c * CHUNK + (uint32_t)j;
                any |= (rr < n && mask[rr] != 0) ? 1 : 0;
            }
        }
        if (!__syncthreads_or(any)) return;
    }
    {
        const float4* src = reinterpret_cast<const float4*>(Wp);
        float4* dst = reinterpret_cast<float4*>(s_w);
        for (int k = threadIdx.x; k < P::TOTAL / 4; k += PB) dst[k] = src[k];
    }
    __syncthreads();
    const int l = threadIdx.x & 63, r16 = l & 15, g = l >> 4;
    float ls[4], sd[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        ls[k] = s_w[P::O_LOGSTD + k];
        sd[k] = __builtin_amdgcn_exp2f(1.4426950408889634f * ls[k]);
    }
    // this lane's standardisation constants (its input indices do not change between chunks)
    // (the k-block constants are re-read from LDS per chunk, CF2_POLICY_STD_LDS: 16 fewer live VGPRs)
#ifndef CF2_POLICY_STD_LDS
#define CF2_POLICY_STD_LDS 1
#endif
    float mean8[P::KB1 > 0 ? P::KB1 : 1][8], scale8[P::KB1 > 0 ? P::KB1 : 1][8], mean1[P::KS1 > 0 ? P::KS1 : 1],
        scale1[P::KS1 > 0 ? P::KS1 : 1], meanr[P::SL ? P::R1 : 1], scaler[P::SL ? P::R1 : 1];
    if constexpr (P::SL)
#pragma unroll
        for (int r = 0; r < P::R1; ++r) {
            meanr[r] = s_w[P::O_MEAN + P::K1R + r];
            scaler[r] = s_w[P::O_SCALE + P::K1R + r];
        }
    const uint32_t g0 = g == 0 ? 0xffffffffu : 0u;      // slot-mode B operand lives in lane group 0
#if !CF2_POLICY_STD_LDS
#pragma unroll
    for (int kb = 0; kb < P::KB1; ++kb)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            mean8[kb][j] = s_w[P::O_MEAN + 32 * kb + 8 * g + j];
            scale8[kb][j] = s_w[P::O_SCALE + 32 * kb + 8 * g + j];
        }
#endif
#pragma unroll
    for (int ks = 0; ks < P::KS1; ++ks) {
        const int k = __builtin_elementwise_min(P::K1R + 4 * ks + g, D - 1);
        mean1[ks] = s_w[P::O_MEAN + k];
        scale1[ks] = s_w[P::O_SCALE + k];
    }
    ObsRegs<D, PREC> X;
    if (MODE == 0 && wave < nchunks) load_obs<D, PREC>(obs, n, wave * CHUNK, l, X);
    for (uint32_t c = wave; c < nchunks; c += nwaves) {
        const uint32_t r0 = c * CHUNK;
        if (MODE == 1) {
            // marked rows are sparse: a chunk without one is skipped before its observations load
            const uint32_t rr = r0 + (uint32_t)l;
            if (!__builtin_amdgcn_ballot_w64(l < CHUNK && rr < n && mask[rr] != 0)) continue;
            load_obs<D, PREC>(obs, n, r0, l, X);
        }
        // the fragments are loop-invariant: without an opaque base the compiler hoists all LDS
        // reads out of the chunk loop and spills them (an integer offset, not a laundered pointer:
        // the reads must stay LDS reads)
        int off = 0;
        asm volatile("" : "+v"(off));
        const float* sw = s_w + off;
        ObsRegs<D, PREC> Xc = X;
#if CF2_POLICY_STD_LDS
#pragma unroll
        for (int kb = 0; kb < P::KB1; ++kb)
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const float4 m = *reinterpret_cast<const float4*>(&sw[P::O_MEAN + 32 * kb + 8 * g + 4 * q]);
                const float4 sc = *reinterpret_cast<const float4*>(&sw[P::O_SCALE + 32 * kb + 8 * g + 4 * q]);
                mean8[kb][4 * q] = m.x; mean8[kb][4 * q + 1] = m.y; mean8[kb][4 * q + 2] = m.z; mean8[kb][4 * q + 3] = m.w;
                scale8[kb][4 * q] = sc.x; scale8[kb][4 * q + 1] = sc.y; scale8[kb][4 * q + 2] = sc.z; scale8[kb][4 * q + 3] = sc.w;
            }
#endif
        // observation standardisation (obs - mean) * scale, per input index of this lane
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
            for (int kb = 0; kb < P::KB1; ++kb)
#pragma unroll
                for (int j = 0; j < 8; ++j) Xc.x8[rt][kb][j] = (Xc.x8[rt][kb][j] - mean8[kb][j]) * scale8[kb][j];
#pragma unroll
            for (int ks = 0; ks < P::KS1; ++ks) Xc.x1[rt][ks] = (Xc.x1[rt][ks] - mean1[ks]) * scale1[ks];
            if constexpr (P::SL)
#pragma unroll
                for (int r = 0; r < P::R1; ++r) Xc.xr[rt][r] = (Xc.xr[rt][r] - meanr[r]) * scaler[r];
        }
        // prefetch the next chunk's observations while this one runs on the matrix cores
        if (MODE == 0 && c + nwaves < nchunks) load_obs<D, PREC>(obs, n, (c + nwaves) * CHUNK, l, X);
        // ---- layer 1: [pi | v] 128 neurons (8 n-tiles); MODE 1 runs only the v half
        constexpr int NT0 = PI ? 0 : 4;
        f4v h1[8][RT];
#pragma unroll
        for (int nt = NT0; nt < 8; ++nt) {
            const f4v b = *reinterpret_cast<const f4v*>(&sw[P::O_BIAS + P::B_L1 + 16 * nt + 4 * g]);
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
        if constexpr (P::SL) {
            bf8v bs[RT];
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                uint16_t hb[P::R1], lb[P::R1];
#pragma unroll
                for (int r = 0; r < P::R1; ++r) {
                    const __bf16 h = (__bf16)Xc.xr[rt][r];
                    hb[r] = __builtin_bit_cast(uint16_t, h);
                    lb[r] = __builtin_bit_cast(uint16_t, (__bf16)(Xc.xr[rt][r] - (float)h));
                }
                u4v wds;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    uint32_t wq = 0;
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        const int sl = 2 * q + e;
                        const uint32_t v = sl < P::R1 ? hb[sl] : sl < 2 * P::R1 ? lb[sl - P::R1]
                                         : sl < 3 * P::R1 ? hb[sl - 2 * P::R1] : 0u;
                        wq |= v << (16 * e);
                    }
                    wds[q] = wq & g0;
                }
                bs[rt] = __builtin_bit_cast(bf8v, wds);
            }
#pragma unroll
            for (int nt = NT0; nt < 8; ++nt) {
                const bf8v a = __builtin_bit_cast(bf8v, *reinterpret_cast<const float4*>(sw + P::O_L1F + nt * P::FS + 4 * l));
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) h1[nt][rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bs[rt], h1[nt][rt], 0, 0, 0);
            }
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
            const f4v bp = *reinterpret_cast<const f4v*>(&sw[P::O_BIAS + P::B_L2P + 16 * nt + 4 * g]);
            const f4v bv = *reinterpret_cast<const f4v*>(&sw[P::O_BIAS + P::B_L2V + 16 * nt + 4 * g]);
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
        // ---- layer 3: one n-tile, rows 0..3 = mu, row 4 = v
        f4v o[RT];
        {
            const f4v b = *reinterpret_cast<const f4v*>(&sw[P::O_BIAS + P::B_L3 + 4 * g]);
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
                    ld_frag(sw, P::O_L3 + (2 * half + kb) * P::FB, l, ah, al);
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
                    const float a = sw[P::O_L3 + ((half ? P::KSP : 0) + ks) * P::FF + l];
#pragma unroll
                    for (int rt = 0; rt < RT; ++rt) o[rt] = mfma4(a, h[t][rt][i], o[rt]);
                }
            }
        }
        // lanes 0..15 hold mu[0..3] of row 16 rt + l, lanes 16..31 hold v in register 0
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const uint32_t row = r0 + 16 * rt + r16;
            if (row >= n) continue;
            if (g == 1 && (MODE == 0 || mask[row])) val[row] = o[rt][0];
            if (PI && g == 0) {
                float eps[4] = {0.0f, 0.0f, 0.0f, 0.0f};
                if (sample) {
                    const Keys K = make_keys(key0, key1);
                    const U4 u = philox(K, 0u, counter, row_offset + row, TAG_POLICY);
                    box_muller(u.x, u.y, eps[0], eps[1]);
                    box_muller(u.z, u.w, eps[2], eps[3]);
                }
                float lp = 0.0f;
                float4 a;
                float* ap = &a.x;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    ap[k] = o[rt][k] + sd[k] * eps[k];
                    lp += -0.5f * eps[k] * eps[k] - ls[k] - 0.91893853320467274f;    // 0.5 log(2 pi)
                }
                reinterpret_cast<float4*>(act)[row] = a;
                if (logp) logp[row] = sample ? lp : 1.0f;
            }
        }
    }
}

static int policy_grid(uint32_t n) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint32_t want = (n + PW * CHUNK - 1) / (PW * CHUNK);
    // resident blocks per CU: LDS (~58-62 KB of fragments per block) and the wave budget
    const uint32_t by_waves = (uint32_t)(4 * CF2_POLICY_WAVES / PW);
#ifndef CF2_POLICY_PER_CU
#define CF2_POLICY_PER_CU 2u     // resident blocks per CU the persistent grid is sized for
#endif
    const uint32_t cap_cu = CF2_POLICY_PER_CU;
    const uint32_t per_cu = by_waves < cap_cu ? (by_waves ? by_waves : 1u) : cap_cu;
    const uint32_t cap = per_cu * (uint32_t)cus;
    return (int)(want < cap ? want : cap);
}

// Batched GAE (algs/core.py:459-535 finish_path per episode slice, with per-env boundaries):
// one thread per env scans the [T, N] buffers backward; loads/stores at step t are coalesced
// over envs.  Bootstraps: terminal 0, time-out trunc_val[t], end of buffer last_val.  Reward
// scaling (core.py:522-529): rew_den > 0 puts clip(r / rew_den, -10, 10) into delta.  disc
// (optional): the per-episode discounted returns of the unscaled rewards (core.py:519).
__global__ void __launch_bounds__(256) gae_kernel(uint32_t T, uint32_t n, const float* __restrict__ rew,
                                                  const float* __restrict__ val, const uint8_t* __restrict__ done,
                                                  const uint8_t* __restrict__ trunc, const float* __restrict__ trunc_val,
                                                  const float* __restrict__ last_val, float gamma, float lam,
                                                  float rew_den, float* __restrict__ adv, float* __restrict__ ret,
                                                  float* __restrict__ disc) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    float nxt_adv = 0.0f, nxt_val = last_val[e], nxt_ret = last_val[e];
    // the backward scan is serial in t; the loads of U steps are issued together so the scan
    // waits for memory once per U steps instead of once per step (the time-out value is read
    // only where an episode timed out)
    constexpr int U = 8;
    for (int t0 = (int)T - 1; t0 >= 0; t0 -= U) {
        float rr[U], vv[U];
        uint8_t dd[U], tt[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int t = t0 - j;
            const size_t k = (size_t)(t < 0 ? 0 : t) * n + e;
            rr[j] = rew[k];
            vv[j] = val[k];
            dd[j] = done[k];
            tt[j] = trunc[k];
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int t = t0 - j;
            if (t < 0) break;
            const size_t k = (size_t)t * n + e;
            const bool d = dd[j] != 0;
            const float boot = d ? (tt[j] ? trunc_val[k] : 0.0f) : nxt_val;
            const float v = vv[j], r = rr[j];
            const float rs = rew_den > 0.0f ? fminf(fmaxf(r / rew_den, -10.0f), 10.0f) : r;
            const float a = (rs + gamma * boot - v) + gamma * lam * (d ? 0.0f : nxt_adv);
            adv[k] = a;
            ret[k] = a + v;
            if (disc) {
                nxt_ret = r + gamma * (d ? boot : nxt_ret);
                disc[k] = nxt_ret;
            }
            nxt_adv = a;
            nxt_val = v;
        }
    }
}

}  // namespace cf2

using namespace cf2;

extern "C" int cf2_gae(uint32_t T, uint32_t n, const float* rew_dev, const float* val_dev, const uint8_t* done_dev,
                       const uint8_t* trunc_dev, const float* trunc_val_dev, const float* last_val_dev, float gamma,
                       float lam, float rew_den, float* adv_dev, float* ret_dev, float* disc_ret_dev, void* stream) {
    if (!rew_dev || !val_dev || !done_dev || !trunc_dev || !trunc_val_dev || !last_val_dev || !adv_dev || !ret_dev)
        return CF2_ERR_INVALID_ARG;
    if (n == 0 || T == 0) return CF2_OK;
    hipLaunchKernelGGL(gae_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, T, n, rew_dev, val_dev,
                       done_dev, trunc_dev, trunc_val_dev, last_val_dev, gamma, lam, rew_den, adv_dev, ret_dev,
                       disc_ret_dev);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? CF2_OK : CF2_ERR_HIP;
}

template <int D, int PREC>
static int policy_launch(const float* packed_dev, uint32_t n, const float* obs_dev, uint32_t k0, uint32_t k1,
                         uint32_t counter, uint32_t row_offset, int sample, float* act_dev, float* val_dev,
                         float* logp_dev, const uint8_t* mask_dev, hipStream_t s) {
    const dim3 grid(policy_grid(n)), block(PB);
    if (mask_dev)
        hipLaunchKernelGGL((policy_kernel<D, PREC, 1>), grid, block, 0, s, packed_dev, n, obs_dev, 0u, 0u, 0u, 0u, 0,
                           nullptr, val_dev, nullptr, mask_dev);
    else
        hipLaunchKernelGGL((policy_kernel<D, PREC, 0>), grid, block, 0, s, packed_dev, n, obs_dev, k0, k1, counter,
                           row_offset, sample, act_dev, val_dev, logp_dev, nullptr);
    return hipGetLastError() == hipSuccess ? CF2_OK : CF2_ERR_HIP;
}

static int policy_dispatch(const float* packed_dev, uint32_t n, uint32_t obs_dim, int precision, const float* obs_dev,
                           uint32_t k0, uint32_t k1, uint32_t counter, uint32_t row_offset, int sample, float* act_dev,
                           float* val_dev, float* logp_dev, const uint8_t* mask_dev, hipStream_t s) {
#define CF2_POLICY_CASE(D_, P_)                                                                                \
    if (obs_dim == D_ && precision == P_)                                                                      \
        return policy_launch<D_, P_>(packed_dev, n, obs_dev, k0, k1, counter, row_offset, sample, act_dev,      \
                                     val_dev, logp_dev, mask_dev, s);
    CF2_POLICY_CASE(34, CF2_POLICY_F32)
    CF2_POLICY_CASE(34, CF2_POLICY_BF16X3)
    CF2_POLICY_CASE(42, CF2_POLICY_F32)
    CF2_POLICY_CASE(42, CF2_POLICY_BF16X3)
#undef CF2_POLICY_CASE
    return CF2_ERR_UNSUPPORTED;
}

static bool policy_shape_ok(uint32_t obs_dim, int precision) {
    return (obs_dim == 34 || obs_dim == 42) && (precision == CF2_POLICY_F32 || precision == CF2_POLICY_BF16X3);
}

extern "C" size_t cf2_policy_weights_count(uint32_t obs_dim) {
    if (obs_dim == 34) return PolicyLayout<34>::TOTAL;
    if (obs_dim == 42) return PolicyLayout<42>::TOTAL;
    return 0;
}

extern "C" size_t cf2_policy_packed_count(uint32_t obs_dim, int precision) {
    if (!policy_shape_ok(obs_dim, precision)) return 0;
    if (obs_dim == 34) return precision == CF2_POLICY_F32 ? Packed<34, CF2_POLICY_F32>::TOTAL : Packed<34, CF2_POLICY_BF16X3>::TOTAL;
    return precision == CF2_POLICY_F32 ? Packed<42, CF2_POLICY_F32>::TOTAL : Packed<42, CF2_POLICY_BF16X3>::TOTAL;
}

extern "C" int cf2_policy_pack(const float* weights_dev, uint32_t obs_dim, int precision, float* packed_dev,
                               void* stream) {
    if (!weights_dev || !packed_dev) return CF2_ERR_INVALID_ARG;
    if (!policy_shape_ok(obs_dim, precision)) return CF2_ERR_UNSUPPORTED;
    if ((uintptr_t)packed_dev & 15u) return CF2_ERR_INVALID_ARG;
    const hipStream_t s = (hipStream_t)stream;
    const uint32_t total = (uint32_t)cf2_policy_packed_count(obs_dim, precision);
    const dim3 grid((total + 255) / 256), block(256);
    if (obs_dim == 34 && precision == CF2_POLICY_F32)
        hipLaunchKernelGGL((pack_kernel<34, CF2_POLICY_F32>), grid, block, 0, s, weights_dev, packed_dev);
    else if (obs_dim == 34)
        hipLaunchKernelGGL((pack_kernel<34, CF2_POLICY_BF16X3>), grid, block, 0, s, weights_dev, packed_dev);
    else if (precision == CF2_POLICY_F32)
        hipLaunchKernelGGL((pack_kernel<42, CF2_POLICY_F32>), grid, block, 0, s, weights_dev, packed_dev);
    else
        hipLaunchKernelGGL((pack_kernel<42, CF2_POLICY_BF16X3>), grid, block, 0, s, weights_dev, packed_dev);
    return hipGetLastError() == hipSuccess ? CF2_OK : CF2_ERR_HIP;
}

extern "C" int cf2_policy_forward(const float* packed_dev, uint32_t n, uint32_t obs_dim, int precision,
                                  const float* obs_dev, uint64_t seed, uint32_t counter, uint32_t row_offset,
                                  int sample, float* act_dev, float* val_dev, float* logp_dev, void* stream) {
    if (!packed_dev || !obs_dev || !act_dev || !val_dev) return CF2_ERR_INVALID_ARG;
    if (!policy_shape_ok(obs_dim, precision)) return CF2_ERR_UNSUPPORTED;
    if (((uintptr_t)obs_dev & 7u) || ((uintptr_t)act_dev & 15u) || ((uintptr_t)packed_dev & 15u))
        return CF2_ERR_INVALID_ARG;
    if (n == 0) return CF2_OK;
    return policy_dispatch(packed_dev, n, obs_dim, precision, obs_dev, (uint32_t)seed, (uint32_t)(seed >> 32), counter,
                           row_offset, sample, act_dev, val_dev, logp_dev, nullptr, (hipStream_t)stream);
}

extern "C" int cf2_value_forward_masked(const float* packed_dev, uint32_t n, uint32_t obs_dim, int precision,
                                        const float* obs_dev, const uint8_t* mask_dev, float* val_dev, void* stream) {
    if (!packed_dev || !obs_dev || !mask_dev || !val_dev) return CF2_ERR_INVALID_ARG;
    if (!policy_shape_ok(obs_dim, precision)) return CF2_ERR_UNSUPPORTED;
    if (((uintptr_t)obs_dev & 7u) || ((uintptr_t)packed_dev & 15u)) return CF2_ERR_INVALID_ARG;
    if (n == 0) return CF2_OK;
    return policy_dispatch(packed_dev, n, obs_dim, precision, obs_dev, 0u, 0u, 0u, 0u, 0, nullptr, val_dev, nullptr,
                           mask_dev, (hipStream_t)stream);
}
