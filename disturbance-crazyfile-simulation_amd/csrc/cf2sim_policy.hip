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
// RT row tiles of 16 rows and prefetches the next chunk's observations while the
// current one runs.  The packed block (A-operand fragments, lane-ordered:
// conflict-free ds_read_b32 / ds_read_b128) is staged into LDS once per block.
//
// Flat weight block (cf2_policy_weights_count floats; input-major so output neurons are contiguous):
//   pi: W1[D][50] b1[50] W2[50][50] b2[50] W3[50][4] b3[4] log_std[4]
//   v:  W1[D][64] b1[64] W2[64][64] b2[64] W3[64]    b3[1]
//   obs standardisation (core.py:383-388, OnlineMeanStd): mean[D], scale[D] = 1 / (std + 1e-5);
//   both networks see (obs - mean) * scale (identity: mean 0, scale 1)
#include "cf2sim_policy.h"

namespace cf2 {

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

// mode: 0 = policy (mu, sample, logp) + value of every row; 1 = value only, rows with mask[r] != 0
template <int D, int PREC, int MODE>
__global__ void __launch_bounds__(PB, POLICY_WAVES) policy_kernel(const float* __restrict__ Wp, uint32_t n,
                                                                      const float* __restrict__ obs, uint32_t key0,
                                                                      uint32_t key1, uint32_t counter,
                                                                      uint32_t row_offset, int sample,
                                                                      float* __restrict__ act, float* __restrict__ val,
                                                                      float* __restrict__ logp,
                                                                      const uint8_t* __restrict__ mask) {
    using P = Packed<D, PREC>;
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
    PolicyLane<D, PREC> C;
    policy_lane_init<D, PREC>(s_w + P::O_BIAS, g, C);
    ObsRegs<D, PREC> X;
    if (MODE == 0 && wave < nchunks) load_obs<D, PREC>(obs, n, wave * CHUNK, l, X);
    // sampling noise, one Philox block per row: at every 4th chunk lane group g draws the rows of
    // the wave's chunk k + g (lane 16 g + r), and chunk k + j takes its rows' normals from lane
    // group j (ds_bpermute), instead of all 64 lanes drawing every chunk's 16 rows
    constexpr bool ROWNOISE = MODE == 0 && RT == 1;
    float ep[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    uint32_t kk = 0;
    for (uint32_t c = wave; c < nchunks; c += nwaves, ++kk) {
        if (ROWNOISE && sample && (kk & 3u) == 0u) {
            const uint32_t cg = c + (uint32_t)g * nwaves;
            if (cg < nchunks) policy_noise(key0, key1, counter, row_offset + cg * CHUNK + (uint32_t)r16, ep);
        }
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
        policy_standardize<D, PREC>(sw + P::O_BIAS, g, C, Xc);
        // prefetch the next chunk's observations while this one runs on the matrix cores
        if (MODE == 0 && c + nwaves < nchunks) load_obs<D, PREC>(obs, n, (c + nwaves) * CHUNK, l, X);
        f4v o[RT];
        policy_layers<D, PREC, MODE>(sw, sw + P::O_BIAS, sw + P::O_L3, l, Xc, o);
        if constexpr (ROWNOISE) {
            float e[4];
            const int src = (int)((((kk & 3u) << 4) | (uint32_t)r16) << 2);
#pragma unroll
            for (int k = 0; k < 4; ++k) e[k] = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(ep[k])));
            const uint32_t row = r0 + (uint32_t)r16;
            if (row < n) policy_emit_eps<D, PREC, MODE>(o[0], row, g, C, e, sample, act, val, logp, mask);
        } else {
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                const uint32_t row = r0 + 16 * rt + r16;
                if (row >= n) continue;
                policy_emit<D, PREC, MODE>(o[rt], row, g, C, key0, key1, counter, row_offset, sample, act, val, logp,
                                           mask);
            }
        }
    }
}

static int policy_grid(uint32_t n) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint32_t want = (n + PW * CHUNK - 1) / (PW * CHUNK);
    // resident blocks per CU: LDS (~58-62 KB of fragments per block) and the wave budget
    const uint32_t by_waves = (uint32_t)(4 * POLICY_WAVES / PW);
    const uint32_t cap_cu = 2u;      // resident blocks per CU the persistent grid is sized for (1: slower)
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
