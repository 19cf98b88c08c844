// cf2sim_policy.hip -- fused Gaussian MLP actor-critic forward for the batched rollout caller
// (SURVEY section 8, row f3).
//
// Restates, for a whole batch in one launch, ActorCritic.step of the reference
// (phoenix_drone_simulation/algs/core.py:371-395) with its PPO networks (algs/ppo/defaults.py:8-13):
//   pi: obs -> Linear(50) -> ReLU -> Linear(50) -> ReLU -> Linear(4) -> mu;  a = mu + exp(log_std) * eps
//       logp = Normal(mu, std).log_prob(a).sum(-1)                           (core.py:228-291)
//   v:  obs -> Linear(64) -> tanh -> Linear(64) -> tanh -> Linear(1)      (MLPCritic)
// As torch runs it, each layer is a separate GEMM plus an activation kernel, with 50- and 64-wide
// activations round-tripping through HBM (~0.6 ms per step at 262k rows).  Here one lane owns
// one row end to end: the obs row is staged through LDS (a block's rows are contiguous), the
// activations never leave VGPRs, and the weights -- identical for every lane -- are scalar loads
// (SGPR operands of packed v_pk_fma_f32, two output neurons per instruction).  fp32 throughout:
// on gfx950 fp32 MFMA issues at the plain-VALU FMA rate, packed VALU at twice it.
//
// Weight block (floats, all matrices input-major so output neurons are contiguous):
//   pi: W1[D][50] b1[50] W2[50][50] b2[50] W3[50][4] b3[4] log_std[4]
//   v:  W1[D][64] b1[64] W2[64][64] b2[64] W3[64]    b3[1]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "cf2sim_rng.h"
#include "../../include/cf2sim.h"

namespace cf2 {

typedef float f2 __attribute__((ext_vector_type(2)));
// weights are read through the constant address space: scalar loads, and provably no alias of
// the private activation arrays (a generic pointer laundered by asm would pin those to scratch)
typedef const __attribute__((address_space(4))) float* cptr;

template <int D>
struct PolicyLayout {
    static constexpr int P_W1 = 0, P_B1 = P_W1 + D * 50, P_W2 = P_B1 + 50, P_B2 = P_W2 + 50 * 50, P_W3 = P_B2 + 50,
                         P_B3 = P_W3 + 50 * 4, P_LOGSTD = P_B3 + 4;
    static constexpr int V_W1 = P_LOGSTD + 4, V_B1 = V_W1 + D * 64, V_W2 = V_B1 + 64, V_B2 = V_W2 + 64 * 64,
                         V_W3 = V_B2 + 64, V_B3 = V_W3 + 64;
    static constexpr int TOTAL = V_B3 + 1;
};

struct W16 { float w[16]; };
__device__ __forceinline__ W16 load16(cptr p, int n) {
    W16 r;
#pragma unroll
    for (int k = 0; k < 16; ++k) r.w[k] = k < n ? p[k] : 0.0f;
    return r;
}

// y[OUT] = b + sum_i W[i][.] x[i]  (W input-major); two outputs per v_pk_fma_f32 with the weight
// pair as an SGPR operand.  The flattened weights are walked in chunks of 16 (one
// s_load_dwordx16), software-pipelined by hand: chunk c+1 is requested before chunk c's FMAs and
// scheduling barriers keep the compiler from hoisting every load of the layer to the top (which
// needs thousands of SGPRs and spills them to VGPR lanes).  A weight pair never straddles an
// input row (OUT is even, chunks start at even flat indices).
#ifndef CF2_POLICY_PREFETCH
#define CF2_POLICY_PREFETCH 3   // chunks of 16 weights in flight ahead of the FMAs (16 SGPRs each)
#endif
constexpr int PF = CF2_POLICY_PREFETCH;

// one chunk of 16 flattened weights; recursion (not a loop) guarantees full unrolling, so the
// input / accumulator indices are compile-time and x[] / acc[] stay in registers.  ring[k] holds
// chunk C + k; the load of chunk C + PF is issued before chunk C's FMAs.
template <int C, int NC, int IN, int OUT>
struct Chunks {
    static __device__ __forceinline__ void run(cptr W, const float* x, f2* acc, const W16 (&ring)[PF]) {
        constexpr int TOT = IN * OUT;
        W16 nring[PF];
#pragma unroll
        for (int k = 0; k + 1 < PF; ++k) nring[k] = ring[k + 1];
        if constexpr (C + PF < NC) nring[PF - 1] = load16(W + 16 * (C + PF), TOT - 16 * (C + PF) < 16 ? TOT - 16 * (C + PF) : 16);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < 16; k += 2) {
            const int f = 16 * C + k;
            if (f < TOT) {
                const int i = f / OUT, j = f % OUT;
                acc[j / 2] = __builtin_elementwise_fma(f2{ring[0].w[k], ring[0].w[k + 1]}, f2{x[i], x[i]}, acc[j / 2]);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (C + 1 < NC) Chunks<C + 1, NC, IN, OUT>::run(W, x, acc, nring);
    }
};

template <int IN, int OUT>
__device__ __forceinline__ void dense(cptr W, cptr b, const float* x, float* y) {
    static_assert(OUT % 2 == 0, "pairs of outputs");
    constexpr int TOT = IN * OUT, NC = (TOT + 15) / 16;
    f2 acc[OUT / 2];
#pragma unroll
    for (int j = 0; j < OUT / 2; ++j) acc[j] = f2{b[2 * j], b[2 * j + 1]};
    W16 ring[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k)
        if (k < NC) ring[k] = load16(W + 16 * k, TOT - 16 * k < 16 ? TOT - 16 * k : 16);
    Chunks<0, NC, IN, OUT>::run(W, x, acc, ring);
#pragma unroll
    for (int j = 0; j < OUT / 2; ++j) { y[2 * j] = acc[j].x; y[2 * j + 1] = acc[j].y; }
}

// tanh(x) = sign(x) (1 - 2 / (exp(2|x|) + 1)) on v_exp_f32 / v_rcp_f32 (abs error < 2e-7)
__device__ __forceinline__ float tanh_fast(float x) {
    const float e = __builtin_amdgcn_exp2f(2.8853900817779268f * fabsf(x));   // exp(2|x|)
    return __builtin_copysignf(1.0f - 2.0f * __builtin_amdgcn_rcpf(e + 1.0f), x);
}

template <int D>
__device__ __forceinline__ float value_net(cptr W, const float* x) {
    using L = PolicyLayout<D>;
    float h1[64], h2[64];
    dense<D, 64>(W + L::V_W1, W + L::V_B1, x, h1);
#pragma unroll
    for (int j = 0; j < 64; ++j) h1[j] = tanh_fast(h1[j]);
    dense<64, 64>(W + L::V_W2, W + L::V_B2, h1, h2);
    float v = W[L::V_B3];
#pragma unroll
    for (int j = 0; j < 64; ++j) v = __builtin_fmaf(W[L::V_W3 + j], tanh_fast(h2[j]), v);
    return v;
}

enum : uint32_t { TAG_POLICY = 3 };

// mode: 0 = policy (mu, sample, logp) + value of every row; 1 = value only, rows with mask[r] != 0
template <int D, int MODE>
__global__ void __launch_bounds__(256) policy_kernel(const float* __restrict__ Wg, uint32_t n,
                                                     const float* __restrict__ obs, uint32_t key0, uint32_t key1,
                                                     uint32_t counter, uint32_t row_offset, int sample,
                                                     float* __restrict__ act, float* __restrict__ val,
                                                     float* __restrict__ logp, const uint8_t* __restrict__ mask) {
    using L = PolicyLayout<D>;
    constexpr uint32_t B = 256;
    const cptr W = (cptr)Wg;
    __shared__ __align__(16) float s_x[B * D];
    const uint32_t tid = threadIdx.x, base = blockIdx.x * B, r = base + tid;
    const uint32_t nvalid = n - base < B ? n - base : B;
    if (MODE == 1) {
        // value-only pass (time-out bootstraps): nothing to do for a block without marked rows
        const int m = r < n ? (int)mask[r] : 0;
        if (!__syncthreads_or(m)) return;
    }
    {   // stage the block's rows (contiguous, 16-B aligned: B * D * 4 is a multiple of 16)
        const float* src = obs + (size_t)base * D;
        if (nvalid == B && (B * D) % 4 == 0) {
            const float4* s4 = reinterpret_cast<const float4*>(src);
            float4* d4 = reinterpret_cast<float4*>(s_x);
            for (uint32_t k = tid; k < B * D / 4; k += B) d4[k] = s4[k];
        } else {
            for (uint32_t k = tid; k < nvalid * D; k += B) s_x[k] = src[k];
        }
    }
    __syncthreads();
    if (r >= n) return;
    if (MODE == 1 && !mask[r]) return;
    // the obs row is read from LDS once per network, so it is not live across the value net
    float x[D];
#pragma unroll
    for (int k = 0; k < D; ++k) x[k] = s_x[tid * D + k];
    const float v = value_net<D>(W, x);
    val[r] = v;
    if (MODE == 1) return;
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < D; ++k) x[k] = s_x[tid * D + k];
    float h1[50], h2[50], mu[4];
    dense<D, 50>(W + L::P_W1, W + L::P_B1, x, h1);
#pragma unroll
    for (int j = 0; j < 50; ++j) h1[j] = fmaxf(h1[j], 0.0f);
    dense<50, 50>(W + L::P_W2, W + L::P_B2, h1, h2);
#pragma unroll
    for (int j = 0; j < 50; ++j) h2[j] = fmaxf(h2[j], 0.0f);
    dense<50, 4>(W + L::P_W3, W + L::P_B3, h2, mu);
    float eps[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (sample) {
        const Keys K = make_keys(key0, key1);
        const U4 u = philox(K, 0u, counter, row_offset + r, TAG_POLICY);
        box_muller(u.x, u.y, eps[0], eps[1]);
        box_muller(u.z, u.w, eps[2], eps[3]);
    }
    float lp = 0.0f;
    float4 a;
    float* ap = &a.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float ls = W[L::P_LOGSTD + k];
        ap[k] = mu[k] + __builtin_amdgcn_exp2f(1.4426950408889634f * ls) * eps[k];
        lp += -0.5f * eps[k] * eps[k] - ls - 0.91893853320467274f;    // 0.5 log(2 pi)
    }
    reinterpret_cast<float4*>(act)[r] = a;
    if (logp) logp[r] = sample ? lp : 1.0f;
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
    for (int t = (int)T - 1; t >= 0; --t) {
        const size_t k = (size_t)t * n + e;
        const bool d = done[k] != 0;
        const float boot = d ? (trunc[k] ? trunc_val[k] : 0.0f) : nxt_val;
        const float v = val[k];
        const float r = rew[k];
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

extern "C" size_t cf2_policy_weights_count(uint32_t obs_dim) {
    if (obs_dim == 34) return PolicyLayout<34>::TOTAL;
    if (obs_dim == 42) return PolicyLayout<42>::TOTAL;
    return 0;
}

extern "C" int cf2_policy_forward(const float* weights_dev, uint32_t n, uint32_t obs_dim, const float* obs_dev,
                                  uint64_t seed, uint32_t counter, uint32_t row_offset, int sample, float* act_dev,
                                  float* val_dev, float* logp_dev, void* stream) {
    if (!weights_dev || !obs_dev || !act_dev || !val_dev) return CF2_ERR_INVALID_ARG;
    if (obs_dim != 34 && obs_dim != 42) return CF2_ERR_UNSUPPORTED;
    if (((uintptr_t)obs_dev & 15u) || ((uintptr_t)act_dev & 15u)) return CF2_ERR_INVALID_ARG;
    if (n == 0) return CF2_OK;
    const dim3 grid((n + 255) / 256), block(256);
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    if (obs_dim == 34)
        hipLaunchKernelGGL((policy_kernel<34, 0>), grid, block, 0, (hipStream_t)stream, weights_dev, n, obs_dev, k0, k1,
                           counter, row_offset, sample, act_dev, val_dev, logp_dev, nullptr);
    else
        hipLaunchKernelGGL((policy_kernel<42, 0>), grid, block, 0, (hipStream_t)stream, weights_dev, n, obs_dev, k0, k1,
                           counter, row_offset, sample, act_dev, val_dev, logp_dev, nullptr);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? CF2_OK : CF2_ERR_HIP;
}

extern "C" int cf2_value_forward_masked(const float* weights_dev, uint32_t n, uint32_t obs_dim, const float* obs_dev,
                                        const uint8_t* mask_dev, float* val_dev, void* stream) {
    if (!weights_dev || !obs_dev || !mask_dev || !val_dev) return CF2_ERR_INVALID_ARG;
    if (obs_dim != 34 && obs_dim != 42) return CF2_ERR_UNSUPPORTED;
    if ((uintptr_t)obs_dev & 15u) return CF2_ERR_INVALID_ARG;
    if (n == 0) return CF2_OK;
    const dim3 grid((n + 255) / 256), block(256);
    if (obs_dim == 34)
        hipLaunchKernelGGL((policy_kernel<34, 1>), grid, block, 0, (hipStream_t)stream, weights_dev, n, obs_dev, 0u, 0u, 0u,
                           0u, 0, nullptr, val_dev, nullptr, mask_dev);
    else
        hipLaunchKernelGGL((policy_kernel<42, 1>), grid, block, 0, (hipStream_t)stream, weights_dev, n, obs_dev, 0u, 0u, 0u,
                           0u, 0, nullptr, val_dev, nullptr, mask_dev);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? CF2_OK : CF2_ERR_HIP;
}
