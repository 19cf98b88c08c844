// cf2sim_exchange.hip -- the multi-GPU observation exchange as deltas.
//
// The north star gathers every rank's observation slab to every rank each env-step (RCCL
// all-gather over xGMI).  A row is [o_{k-1}, A0, o_k, A1] (compute_history, envs/base.py:305-321):
// of its 34 floats only o_k (13) is new each step -- o_{k-1} was o_k of the previous step's row,
// and the action slots are actions the receiver issued -- except around auto-resets.  So each
// rank sends, per env-step:
//   * o_k of every env                                   (OL words per env)
//   * a bitmap of the envs that auto-reset this step     (1 bit per env)
//   * for those envs (up to `cap`): the reset row's o_0 and its action part A (the reset's
//     action-buffer entry, A_0 = A_1)                    (1 + OL + 4 words each)
// Receivers keep what they gathered (compact): per env-step they only advance every env's `age`
// (env-steps since its last reset; uint16, saturating; cf2_obs_consume), and a row is materialised
// on request (cf2_obs_rows) from the gathered buffers of step k and k - 1, the age and the actions
// of steps k, k - 1 and k - 2, following the reference's history aliasing (compute_history with the
// action deque holding the action buffer's last entry right after a reset, envs/base.py:455-462;
// the kernel's halias flags):
//   age 0:  [o_0, A, o_k, A]                         (the reset's side entry; o_k from step k)
//   age 1:  [o_{k-1}, a_k, o_k, a_k]                 (both history slots alias the action buffer,
//                                                     which after the step holds a_k in every row:
//                                                     aggregate_phy_steps is a multiple of buf_size,
//                                                     as in the reference's default env)
//   age 2:  [o_{k-1}, a_k, o_k, a_{k-1}]
//   age 3+: [o_{k-1}, a_{k-2}, o_k, a_{k-1}]
// where a_k is the action of the env-step that produced the row and o_{k-1} is o_k of step k - 1.
// The receiver tracks age from the bitmaps (exact: reset or not is always known).  A rank with more
// resets than its side slab holds in one step (an overflow) marks the 64-env pack blocks whose
// resets past their quota got no spill slot (PACK_DROPPED in the block table): exactly those reset
// rows get NaN in their o_0 / A parts and every such block is counted; their o_k parts and all other
// rows stay exact, and the following steps are exact again.
// The capacity may change from step to step (the caller sizes the all-gather): TimeLimit
// truncations are predictable, so the receiver counts, per rank, the envs whose age reaches
// max_steps - L this step -- at most that many time out L steps later (fewer if they crash first)
// -- into pred[step % npred][rank], and the caller adds that count to the crash budget of step
// + L.  Every rank holds the same ages, so every rank derives the same capacity.
//
// The packed buffer's layout and its side-slot allocation: cf2sim_pack.h.
//
// Driving it (cf2_xchg_*): an RCCL communicator of the library's own and, on an exchange stream
// forked from the env stream, one all-gather + one consume per batch of env-steps: eagerly one C
// call per step (cf2_xchg_publish / cf2_xchg_env_step: batches of one), or cf2_xchg_run, whose
// env-steps (the pack fused in, cf2_step_packed) go back to back on the env stream while the
// previous batch's all-gather runs, so neither the host's per-step issue work nor a per-step
// collective bounds the pipeline.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <dlfcn.h>
#include <stdint.h>
#include <string.h>
#include <math.h>
#include <stdlib.h>
#include <chrono>
#include <mutex>
#include <vector>
#include "../../include/cf2sim.h"
#include "cf2sim_internal.h"
#include "cf2sim_pack.h"

namespace cf2 {

constexpr uint32_t XB = 256;        // rows per block of the exchange kernels (4 pack blocks)

// Coalesced copy of `count` floats (16-B aligned, a multiple of 4) between global memory and LDS,
// all threads of the block; the scalar form for a ragged tail block
__device__ __forceinline__ void rows_to_lds(float* s, const float* g, uint32_t count, bool al) {
    if (al && (count & 3u) == 0) {
        const float4* g4 = reinterpret_cast<const float4*>(g);
        float4* s4 = reinterpret_cast<float4*>(s);
        for (uint32_t k = threadIdx.x; k < count / 4u; k += XB) s4[k] = g4[k];
    } else {
        for (uint32_t k = threadIdx.x; k < count; k += XB) s[k] = g[k];
    }
}
__device__ __forceinline__ void lds_to_rows(float* g, const float* s, uint32_t count, bool al) {
    if (al && (count & 3u) == 0) {
        float4* g4 = reinterpret_cast<float4*>(g);
        const float4* s4 = reinterpret_cast<const float4*>(s);
        for (uint32_t k = threadIdx.x; k < count / 4u; k += XB) g4[k] = s4[k];
    } else {
        for (uint32_t k = threadIdx.x; k < count; k += XB) g[k] = s[k];
    }
}

// Sender: one thread per env of this rank (OL: 13 with sensor noise, 17 without).  The block's obs
// rows are read coalesced into LDS, o_k extracted into an LDS stage and written as one contiguous
// run of the o_k slab; the reset bitmap comes from wave ballots; each wave is one pack block, whose
// resets past its quota take spill slots with one pack_alloc (cf2sim_pack.h).  next_scratch: the counters of
// the buffer the next pack on this stream uses (zeroed here; this pack's were zeroed by the last).
template <uint32_t OL>
__global__ void __launch_bounds__(XB) obs_pack_kernel(const float* __restrict__ obs, const uint8_t* __restrict__ reset,
                                                      PackLayout L, uint32_t* __restrict__ pk,
                                                      uint32_t* __restrict__ scratch,
                                                      uint32_t* __restrict__ next_scratch) {
    constexpr uint32_t OD = 2u * (OL + 4u);
    __shared__ __align__(16) float s_rows[XB * OD];
    __shared__ __align__(16) float s_o[XB * OL];
    const uint32_t tid = threadIdx.x, base = blockIdx.x * XB, i = base + tid, lane = tid & 63u;
    const uint32_t nrow = L.n - base < XB ? L.n - base : XB;
    if (blockIdx.x == 0) {
        if (tid == 0) { pk[0] = 0u; pk[1] = L.n; pk[2] = OL; pk[3] = L.cap; }
        if (next_scratch)
            for (uint32_t k = tid; k < PACK_SCRATCH_WORDS; k += XB) next_scratch[k] = 0u;
    }
    const bool live = tid < nrow;
    const bool r = live && reset[i] != 0;
    const uint64_t m = __ballot(r);
    rows_to_lds(s_rows, obs + (size_t)base * OD, nrow * OD, ((uintptr_t)obs & 15u) == 0 && (base * OD) % 4u == 0);
    uint32_t* bits = pk + L.bits();
    const uint32_t wbase = base + (tid & ~63u);
    if (lane == 0 && wbase < L.n) bits[wbase / 32u] = (uint32_t)m;
    if (lane == 32 && wbase + 32u < L.n) bits[wbase / 32u + 1u] = (uint32_t)(m >> 32);
    uint32_t first = 0;
    if (lane == 0 && wbase < L.n) {
        first = m ? pack_alloc(L, scratch, (uint32_t)__popcll(m)) : 0u;
        pk[L.btab() + wbase / XB_PACK] = first;
    }
    first = __shfl(first, 0);
    __syncthreads();
    const float* row = s_rows + tid * OD;
    if (live) {
#pragma unroll
        for (uint32_t k = 0; k < OL; ++k) s_o[tid * OL + k] = row[OL + 4u + k];
    }
    const uint32_t slot = pack_entry_slot(L, wbase / XB_PACK, (uint32_t)__popcll(m & ((1ull << lane) - 1ull)), first);
    if (r && slot != PACK_DROPPED) {
        uint32_t* e = pk + L.side() + slot * L.entry();
        e[0] = i;
        float* ef = reinterpret_cast<float*>(e + 1);
#pragma unroll
        for (uint32_t k = 0; k < OL + 4u; ++k) ef[k] = row[k];     // o_0 and A (= A_0)
    }
    __syncthreads();
    lds_to_rows(reinterpret_cast<float*>(pk + L.o_slab()) + (size_t)base * OL, s_o, nrow * OL,
                ((uintptr_t)pk & 15u) == 0 && (base * OL) % 4u == 0);
}

// Receiver: the steps [k, k + steps) of one consume call (up to CONSUME_MAX: the eager path
// consumes each step, cf2_xchg_run a batch in launches of up to CONSUME_MAX steps).  One thread per global env (rank
// r = i / n) advances the env's age through the steps from its rank's reset bitmaps.  Time-out
// look-ahead: envs whose new age is watch_age at step s are counted per rank into pred[s] (one
// atomic per wave where the wave holds one rank's envs); block 0 zeroes the zero[] rows (the
// counts of the steps after these).  Every pack block whose resets got no side slot is counted
// in overflow.
constexpr uint32_t CONSUME_MAX = 16;
// The steps of one consume launch, as offsets from its first packed buffer (a batch's steps sit
// step_words apart within each rank's run, ranks rank_stride apart) and ring rows (round 5 passed
// CONSUME_MAX pointers of each kind by value: a 456-byte argument block for a one-step consume)
struct ConsumeSteps {
    const uint32_t* pk0;                   // gathered packed buffer of the first step, rank 0
    uint32_t step_words, rank_stride, steps;
    uint32_t* ring;                        // look-ahead counts [npred][world] (null: not counted), or
    uint32_t npred, row0;                  //   step s counts into row (row0 + s) % npred; then the
    uint32_t nzero;                        //   nzero rows after the last step are zeroed
    uint32_t* pred_one;                    // (ring null) the standalone consume's explicit count row
    uint32_t* zero_one;                    //   and the one row it zeroes, or null
    uint32_t* scratch;                     // the batch's spill counters to zero (its packs are done), or null
    uint32_t scratch_words;
};
// (the step loops are unrolled: every step's bitmap word and block-table word are loaded before
// the dependent chain)
__global__ void __launch_bounds__(256) obs_consume_kernel(ConsumeSteps S, uint32_t world, PackLayout L,
                                                          uint16_t* __restrict__ age, uint32_t* __restrict__ overflow,
                                                          uint32_t watch_age) {
    const uint32_t tid = threadIdx.x, total = world * L.n;
    const uint32_t i = blockIdx.x * 256u + tid;
    if (blockIdx.x == 0 && tid < world) {
        if (S.ring) {
            const uint32_t last = S.row0 + S.steps - 1u;
            for (uint32_t z = 0; z < S.nzero; ++z) S.ring[((last + 1u + z) % S.npred) * world + tid] = 0u;
        } else if (S.zero_one) {
            S.zero_one[tid] = 0u;
        }
    }
    if (blockIdx.x == 0 && S.scratch)
        for (uint32_t k = tid; k < S.scratch_words; k += 256u) S.scratch[k] = 0u;
    const bool live = i < total;
    const uint32_t ic = live ? i : total - 1u;
    const uint32_t r = ic / L.n, li = ic - r * L.n;
    const uint32_t r0 = __shfl(r, 0), r63 = __shfl(r, 63);
    const bool head = live && li % XB_PACK == 0;
    const uint32_t* pr = S.pk0 + (size_t)r * S.rank_stride;
    uint32_t bw[CONSUME_MAX], bt[CONSUME_MAX];
#pragma unroll
    for (uint32_t s = 0; s < CONSUME_MAX; ++s) {
        bw[s] = 0u;
        bt[s] = 0u;
        if (s < S.steps) {
            const uint32_t* pk = pr + (size_t)s * S.step_words;
            bw[s] = pk[L.bits() + li / 32u];
            if (head) bt[s] = pk[L.btab() + li / XB_PACK];
        }
    }
    const bool counting = S.ring || S.pred_one;
    uint32_t a = age[ic];
#pragma unroll
    for (uint32_t s = 0; s < CONSUME_MAX; ++s) {
        if (s >= S.steps) break;
        const bool rs = (bw[s] >> (li % 32u)) & 1u;
        a = rs ? 0u : (a < 0xFFFFu ? a + 1u : 0xFFFFu);
        if (counting) {
            uint32_t* row = S.ring ? S.ring + ((S.row0 + s) % S.npred) * world : S.pred_one;
            const bool hit = live && a == watch_age;
            if (r0 == r63) {
                const uint64_t m = __ballot(hit);
                if ((tid & 63u) == 0 && m) atomicAdd(row + r0, (uint32_t)__popcll(m));
            } else if (hit) {
                atomicAdd(row + r, 1u);
            }
        }
        if (overflow && head && bt[s] == PACK_DROPPED) atomicAdd(overflow, 1u);
    }
    if (live) age[ic] = (uint16_t)a;
}

// Rows on request: rows [row0, row0 + nrows) of the global slab of step k, from the gathered
// buffers of step k (pk_all, capacity L.cap, rank r's at r * stride) and k - 1 (pk_prev_all, Lp.cap,
// stride_prev), the ages after step
// k's consume and the actions of steps k, k - 1, k - 2 ([world n, 4] each).  Each thread builds its
// row in LDS, the block writes them out coalesced.  A reset row finds its side entry from its rank
// among its pack block's resets (the bitmap) and the block table (pack_slot).
template <uint32_t OL>
__global__ void __launch_bounds__(XB) obs_rows_kernel(const uint32_t* __restrict__ pk_all, PackLayout L, uint32_t stride,
                                                      const uint32_t* __restrict__ pk_prev_all, PackLayout Lp,
                                                      uint32_t stride_prev, uint32_t world,
                                                      const uint16_t* __restrict__ age,
                                                      const float* __restrict__ a_k, const float* __restrict__ a_km1,
                                                      const float* __restrict__ a_km2, uint32_t row0, uint32_t nrows,
                                                      float* __restrict__ out) {
    constexpr uint32_t OD = 2u * (OL + 4u);
    __shared__ __align__(16) float s_rows[XB * OD];
    __shared__ __align__(16) float s_ok[XB * OL], s_op[XB * OL];
    const uint32_t tid = threadIdx.x, base = blockIdx.x * XB;
    const uint32_t cnt = nrows - base < XB ? nrows - base : XB;
    const bool live = tid < cnt;
    const uint32_t i = row0 + base + (live ? tid : cnt - 1u);
    const uint32_t r = i / L.n, li = i - r * L.n;
    const uint32_t* pk = pk_all + (size_t)r * stride;
    const float* okp = reinterpret_cast<const float*>(pk + L.o_slab()) + (size_t)li * OL;
    const float* opp = reinterpret_cast<const float*>(pk_prev_all + (size_t)r * stride_prev + Lp.o_slab()) + (size_t)li * OL;
    // the block's o_k and o_{k-1} runs staged through LDS with coalesced loads when its rows sit in
    // one rank (a thread's own 13-float run would take 13 loads 52 B apart)
    const uint32_t g0 = row0 + base, rf = g0 / L.n;
    const bool staged = (g0 + cnt - 1u) / L.n == rf;
    if (staged) {
        const uint32_t li0 = g0 - rf * L.n;
        const float* ok0 = reinterpret_cast<const float*>(pk_all + (size_t)rf * stride + L.o_slab()) + (size_t)li0 * OL;
        const float* op0 =
            reinterpret_cast<const float*>(pk_prev_all + (size_t)rf * stride_prev + Lp.o_slab()) + (size_t)li0 * OL;
        rows_to_lds(s_ok, ok0, cnt * OL, ((uintptr_t)ok0 & 15u) == 0);
        rows_to_lds(s_op, op0, cnt * OL, ((uintptr_t)op0 & 15u) == 0);
    }
    __syncthreads();
    const float* okv = staged ? s_ok + tid * OL : okp;
    const float* opv = staged ? s_op + tid * OL : opp;
    const bool rs = (pk[L.bits() + li / 32u] >> (li % 32u)) & 1u;
    const uint32_t a = age[i];
    float* row = s_rows + tid * OD;
    if (live) {
#pragma unroll
        for (uint32_t k = 0; k < OL; ++k) row[OL + 4u + k] = okv[k];
        if (rs) {
            const uint32_t slot = pack_slot(pk, L, li);
            if (slot == PACK_DROPPED) {     // past its block's quota, and the spill area was full
#pragma unroll
                for (uint32_t k = 0; k < OL + 4u; ++k) row[k] = __builtin_nanf("");
#pragma unroll
                for (uint32_t k = 0; k < 4u; ++k) row[2u * OL + 4u + k] = __builtin_nanf("");
            } else {
                const float* ef = reinterpret_cast<const float*>(pk + L.side() + slot * L.entry() + 1u);
#pragma unroll
                for (uint32_t k = 0; k < OL + 4u; ++k) row[k] = ef[k];                    // o_0 and A
#pragma unroll
                for (uint32_t k = 0; k < 4u; ++k) row[2u * OL + 4u + k] = ef[OL + k];    // A_1 = A_0
            }
        } else {
            const float4 ak = reinterpret_cast<const float4*>(a_k)[i];
            const float4 a1 = reinterpret_cast<const float4*>(a_km1)[i];
            const float4 a0 = a >= 3u ? reinterpret_cast<const float4*>(a_km2)[i] : ak;
            const float4 h1 = a == 1u ? ak : a1;
#pragma unroll
            for (uint32_t k = 0; k < OL; ++k) row[k] = opv[k];
            row[OL] = a0.x; row[OL + 1u] = a0.y; row[OL + 2u] = a0.z; row[OL + 3u] = a0.w;
            row[2u * OL + 4u] = h1.x; row[2u * OL + 5u] = h1.y; row[2u * OL + 6u] = h1.z; row[2u * OL + 7u] = h1.w;
        }
    }
    __syncthreads();
    lds_to_rows(out + (size_t)base * OD, s_rows, cnt * OD, ((uintptr_t)out & 15u) == 0 && (base * OD) % 4u == 0);
}

}  // namespace cf2

using namespace cf2;

static bool layout_ok(uint32_t n, uint32_t ol, uint32_t cap) {
    return n > 0 && (ol == 13u || ol == 17u) && cap <= n && (uint64_t)n * (ol + 10u) < (1ull << 31);
}

extern "C" size_t cf2_obs_packed_words(uint32_t n, uint32_t obs_len, uint32_t cap) {
    if (!layout_ok(n, obs_len, cap)) return 0;
    return PackLayout{n, obs_len, cap}.words();
}

extern "C" int cf2_obs_pack(const float* obs_dev, const uint8_t* reset_dev, uint32_t n, uint32_t obs_len, uint32_t cap,
                            uint32_t* packed_dev, uint32_t* scratch_dev, uint32_t* next_scratch_dev, void* stream) {
    if (!obs_dev || !reset_dev || !packed_dev || !scratch_dev || !layout_ok(n, obs_len, cap)) return CF2_ERR_INVALID_ARG;
    if (((uintptr_t)obs_dev & 7u) || ((uintptr_t)packed_dev & 15u) || ((uintptr_t)scratch_dev & 3u)) return CF2_ERR_INVALID_ARG;
    if (next_scratch_dev == scratch_dev) return CF2_ERR_INVALID_ARG;     // this pack counts in its scratch
    const PackLayout L{n, obs_len, cap};
    if (obs_len == 13u)
        hipLaunchKernelGGL(obs_pack_kernel<13>, dim3((n + XB - 1) / XB), dim3(XB), 0, (hipStream_t)stream, obs_dev,
                           reset_dev, L, packed_dev, scratch_dev, next_scratch_dev);
    else
        hipLaunchKernelGGL(obs_pack_kernel<17>, dim3((n + XB - 1) / XB), dim3(XB), 0, (hipStream_t)stream, obs_dev,
                           reset_dev, L, packed_dev, scratch_dev, next_scratch_dev);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? CF2_OK : hip_fail(e);
}

// The look-ahead ring to the host: one block of lanes storing into the pinned host buffer through
// its device mapping.  hipMemcpyAsync device -> pinned host held the calling thread until the copy
// had run (ROCm 7 on MI355X: the next batch's first env-step started 18 us after the exchange's end,
// gpurun_out/r05f trace), which serialised each batch behind the previous exchange; kernel stores
// to the mapped buffer leave the host thread free.
__global__ void __launch_bounds__(256) words_to_host_kernel(const uint32_t* __restrict__ src, uint32_t* dst,
                                                             uint32_t n) {
    for (uint32_t i = threadIdx.x; i < n; i += 256u) dst[i] = src[i];
}

static int words_to_host(const uint32_t* src_dev, uint32_t* dst_host, uint32_t n, hipStream_t st) {
    void* dp = nullptr;
    hipError_t e = hipHostGetDevicePointer(&dp, dst_host, 0);
    if (e != hipSuccess || !dp) {                 // not a mapped pinned buffer: the runtime's copy
        (void)hipGetLastError();
        e = hipMemcpyAsync(dst_host, src_dev, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost, st);
        return e == hipSuccess ? CF2_OK : hip_fail(e);
    }
    hipLaunchKernelGGL(words_to_host_kernel, dim3(1), dim3(256), 0, st, src_dev, (uint32_t*)dp, n);
    e = hipGetLastError();
    return e == hipSuccess ? CF2_OK : hip_fail(e);
}

static int consume_launch(const ConsumeSteps& S, uint32_t world, const PackLayout& L, uint16_t* age, uint32_t* overflow,
                          uint32_t watch_age, hipStream_t st) {
    const uint32_t total = world * L.n;
    hipLaunchKernelGGL(obs_consume_kernel, dim3((total + 255u) / 256u), dim3(256), 0, st, S, world, L, age, overflow,
                       watch_age);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? CF2_OK : hip_fail(e);
}

extern "C" int cf2_obs_consume(const uint32_t* packed_all_dev, uint32_t world, uint32_t n, uint32_t obs_len,
                               uint32_t cap, uint16_t* age_dev, uint32_t* overflow_dev, uint32_t watch_age,
                               uint32_t* pred_dev, uint32_t* pred_next_dev, void* stream) {
    if (!packed_all_dev || !age_dev || world == 0 || world > 256 || !layout_ok(n, obs_len, cap) ||
        (uint64_t)world * n >= (1ull << 31))
        return CF2_ERR_INVALID_ARG;
    if (pred_dev && pred_dev == pred_next_dev) return CF2_ERR_INVALID_ARG;
    if (((uintptr_t)packed_all_dev & 15u) || ((uintptr_t)age_dev & 1u)) return CF2_ERR_INVALID_ARG;
    const PackLayout L{n, obs_len, cap};
    ConsumeSteps S;
    memset(&S, 0, sizeof(S));
    S.pk0 = packed_all_dev; S.step_words = L.words(); S.rank_stride = L.words(); S.steps = 1;
    S.pred_one = pred_dev; S.zero_one = pred_next_dev;
    return consume_launch(S, world, L, age_dev, overflow_dev, watch_age, (hipStream_t)stream);
}

extern "C" int cf2_obs_rows(const uint32_t* packed_all_dev, uint32_t cap, uint32_t stride,
                            const uint32_t* packed_prev_all_dev, uint32_t cap_prev, uint32_t stride_prev,
                            uint32_t world, uint32_t n, uint32_t obs_len, const uint16_t* age_dev, const float* act_dev,
                            const float* act_prev_dev, const float* act_prev2_dev, uint32_t row0, uint32_t nrows,
                            float* rows_dev, void* stream) {
    if (!packed_all_dev || !packed_prev_all_dev || !age_dev || !act_dev || !act_prev_dev || !act_prev2_dev ||
        !rows_dev || world == 0 || !layout_ok(n, obs_len, cap) || !layout_ok(n, obs_len, cap_prev) ||
        (uint64_t)world * n >= (1ull << 31) || (uint64_t)row0 + nrows > (uint64_t)world * n)
        return CF2_ERR_INVALID_ARG;
    const PackLayout L{n, obs_len, cap}, Lp{n, obs_len, cap_prev};
    if (stride == 0) stride = L.words();
    if (stride_prev == 0) stride_prev = Lp.words();
    if ((world > 1 && (stride < L.words() || stride_prev < Lp.words())) || (stride & 3u) || (stride_prev & 3u))
        return CF2_ERR_INVALID_ARG;
    if (((uintptr_t)packed_all_dev & 15u) || ((uintptr_t)packed_prev_all_dev & 15u) || ((uintptr_t)act_dev & 15u) ||
        ((uintptr_t)act_prev_dev & 15u) || ((uintptr_t)act_prev2_dev & 15u) || ((uintptr_t)rows_dev & 3u) ||
        ((uintptr_t)age_dev & 1u))
        return CF2_ERR_INVALID_ARG;
    if (nrows == 0) return CF2_OK;
    const dim3 grid((nrows + XB - 1) / XB);
    if (obs_len == 13u)
        hipLaunchKernelGGL(obs_rows_kernel<13>, grid, dim3(XB), 0, (hipStream_t)stream, packed_all_dev, L, stride,
                           packed_prev_all_dev, Lp, stride_prev, world, age_dev, act_dev, act_prev_dev, act_prev2_dev,
                           row0, nrows, rows_dev);
    else
        hipLaunchKernelGGL(obs_rows_kernel<17>, grid, dim3(XB), 0, (hipStream_t)stream, packed_all_dev, L, stride,
                           packed_prev_all_dev, Lp, stride_prev, world, age_dev, act_dev, act_prev_dev, act_prev2_dev,
                           row0, nrows, rows_dev);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? CF2_OK : hip_fail(e);
}

// ---- the exchange driven natively (cf2_xchg_*): RCCL bound at run time (dlopen), so the library
// needs no link-time RCCL and shares the instance a host framework already loaded
namespace {
struct RcclApi {
    decltype(&ncclGetUniqueId) get_id = nullptr;
    decltype(&ncclCommInitRank) init = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
};
RcclApi g_rccl;
std::mutex g_rccl_mu;
constexpr uint32_t XCHG_MAX_DEPTH = 8, XCHG_MAX_PRED = 1024, XCHG_MAX_BATCH = 64;
// host-time parts: 0 a whole cf2_xchg_run / env_step call, 1 begin (region take), 2 the env-step
// launches, 3 fork event + stream wait, 4 ncclAllGather, 5 consume launches, 6 the closing events
// and the count copy
constexpr int XCHG_HOST_PARTS = 7;
constexpr uint32_t XCHG_MAX_COPIES = 64;
}  // namespace

// Buffers (cf2_xchg_register): `depth` regions, each holding the packed buffers of one batch of up
// to kmax env-steps.  A batch of nb steps at capacity cap packs step s of the batch into
// send[region][s * words(cap)], so the batch is one contiguous run of nb * words(cap) words that one
// all-gather moves: recv[region] then holds [world][nb][words(cap)].  Each publish / batch takes the
// next region (a counter), so the previous step's buffers are always intact for cf2_obs_rows.
struct cf2_xchg {
    ncclComm_t comm;
    uint32_t world, rank, depth;
    int device;
    hipStream_t xs;                    // the exchange stream
    hipEvent_t fork;                   // env stream -> exchange stream
    hipEvent_t free_[XCHG_MAX_DEPTH];  // the all-gather of region q's last batch is done: q may be rewritten
    hipEvent_t last;                   // the end of the latest exchange (its free_ or its count copy's event)
    bool free_rec[XCHG_MAX_DEPTH], end_rec;
    // the count copies to host buffers: per buffer, the event after its latest copy (cf2_xchg_copy_sync)
    uint32_t* copy_host[XCHG_MAX_COPIES];
    hipEvent_t copy_ev[XCHG_MAX_COPIES];
    uint32_t ncopy;
    // inline exchanges not yet ordered before other streams: the stream they ran on
    bool inl;
    hipStream_t inl_stream;
    hipEvent_t inl_ev;
    uint64_t next_region;
    // a batch opened by cf2_xchg_begin and filled by cf2_xchg_step (actions given one env-step at a time)
    bool open;
    uint32_t open_region, open_cap, open_steps;
    // registered buffers
    bool registered;
    uint32_t n, ol, watch, npred, kmax;
    size_t wmax;                       // words of the largest packed buffer (cap = n)
    float* obs[XCHG_MAX_DEPTH];
    uint8_t* done[XCHG_MAX_DEPTH];
    uint32_t* send;                    // [depth][kmax][wmax], then [depth * kmax][PACK_SCRATCH_WORDS] counters
    uint32_t* recv;                    // [depth][world * kmax * wmax]
    uint16_t* age;
    uint32_t* overflow;
    uint32_t* pred;                    // [npred][world]
    // host time per part of the exchange's C calls (CF2_XCHG_HOST_TIMING=1 at create: diagnostics,
    // cf2_xchg_host_times): ns summed over calls, then the call count
    bool timing;
    double host_ns[XCHG_HOST_PARTS];
    uint64_t host_calls;
};

namespace {
struct HostClock {      // accumulates the host time of one part of an exchange call into x->host_ns[part]
    cf2_xchg* x;
    int part;
    std::chrono::steady_clock::time_point t0;
    HostClock(cf2_xchg* x_, int part_) : x(x_), part(part_) { if (x->timing) t0 = std::chrono::steady_clock::now(); }
    ~HostClock() {
        if (x->timing) x->host_ns[part] += std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count();
    }
};
}  // namespace

extern "C" int cf2_xchg_bind(const char* rccl_path) {
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    if (g_rccl.all_gather) return CF2_OK;
    const char* path = rccl_path ? rccl_path : "librccl.so.1";
    void* h = dlopen(path, RTLD_NOW | RTLD_NOLOAD);       // already in the process: that instance
    if (!h) h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) return CF2_ERR_UNSUPPORTED;
    RcclApi a;
    a.get_id = reinterpret_cast<decltype(a.get_id)>(dlsym(h, "ncclGetUniqueId"));
    a.init = reinterpret_cast<decltype(a.init)>(dlsym(h, "ncclCommInitRank"));
    a.all_gather = reinterpret_cast<decltype(a.all_gather)>(dlsym(h, "ncclAllGather"));
    a.destroy = reinterpret_cast<decltype(a.destroy)>(dlsym(h, "ncclCommDestroy"));
    if (!a.get_id || !a.init || !a.all_gather || !a.destroy) return CF2_ERR_UNSUPPORTED;
    g_rccl = a;
    return CF2_OK;
}

extern "C" int cf2_xchg_unique_id(uint8_t* id_out, size_t id_len) {
    if (!id_out || id_len < sizeof(ncclUniqueId)) return CF2_ERR_INVALID_ARG;
    if (!g_rccl.get_id) return CF2_ERR_UNSUPPORTED;
    ncclUniqueId id;
    if (g_rccl.get_id(&id) != ncclSuccess) return CF2_ERR_HIP;
    memcpy(id_out, &id, sizeof(id));
    return CF2_OK;
}

static void xchg_free_events(cf2_xchg* x) {
    if (x->fork) (void)hipEventDestroy(x->fork);
    if (x->inl_ev) (void)hipEventDestroy(x->inl_ev);
    for (uint32_t k = 0; k < XCHG_MAX_DEPTH; ++k)
        if (x->free_[k]) (void)hipEventDestroy(x->free_[k]);
    for (uint32_t k = 0; k < x->ncopy; ++k)
        if (x->copy_ev[k]) (void)hipEventDestroy(x->copy_ev[k]);
    if (x->xs) (void)hipStreamDestroy(x->xs);
}

extern "C" int cf2_xchg_create(const uint8_t* id, size_t id_len, uint32_t world, uint32_t rank, uint32_t depth,
                               cf2_xchg** out) {
    // depth >= 2: the rows of step k are built from the gathered buffers of steps k and k - 1
    if (!id || id_len < sizeof(ncclUniqueId) || !out || world == 0 || world > 256 || rank >= world || depth < 2 ||
        depth > XCHG_MAX_DEPTH)
        return CF2_ERR_INVALID_ARG;
    if (!g_rccl.init) return CF2_ERR_UNSUPPORTED;
    *out = nullptr;
    cf2_xchg* x = new cf2_xchg();
    x->world = world; x->rank = rank; x->depth = depth;
    const char* tv = getenv("CF2_XCHG_HOST_TIMING");
    x->timing = tv && tv[0] == '1';
    hipError_t e = hipGetDevice(&x->device);
    // the exchange stream at the highest priority: streams of different priority get hardware
    // queues of their own, so the exchange runs beside the env-steps instead of queued behind them
    // (at equal priority it shared the env stream's queue: r05d trace)
    int lo_prio = 0, hi_prio = 0;
    if (e == hipSuccess) e = hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio);
    // (a low or the default priority measured the same per env-step: gpurun_out/r05o)
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&x->xs, hipStreamNonBlocking, hi_prio);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&x->fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&x->inl_ev, hipEventDisableTiming);
    for (uint32_t k = 0; e == hipSuccess && k < depth; ++k)
        e = hipEventCreateWithFlags(&x->free_[k], hipEventDisableTiming);
    if (e != hipSuccess) {
        xchg_free_events(x);
        delete x;
        return hip_fail(e);
    }
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    if (g_rccl.init(&x->comm, (int)world, uid, (int)rank) != ncclSuccess) {
        xchg_free_events(x);
        delete x;
        return CF2_ERR_HIP;
    }
    *out = x;
    return CF2_OK;
}

extern "C" int cf2_xchg_destroy(cf2_xchg* x) {
    if (!x) return CF2_OK;
    int st = CF2_OK;
    (void)hipSetDevice(x->device);
    (void)hipStreamSynchronize(x->xs);
    if (g_rccl.destroy && g_rccl.destroy(x->comm) != ncclSuccess) st = CF2_ERR_HIP;
    xchg_free_events(x);
    delete x;
    return st;
}

extern "C" size_t cf2_xchg_send_words(uint32_t n, uint32_t obs_len, uint32_t depth, uint32_t kmax) {
    if (!layout_ok(n, obs_len, n) || depth < 2 || depth > XCHG_MAX_DEPTH || kmax == 0 || kmax > XCHG_MAX_BATCH) return 0;
    return (size_t)depth * kmax * (PackLayout{n, obs_len, n}.words() + PACK_SCRATCH_WORDS);
}

extern "C" size_t cf2_xchg_recv_words(uint32_t n, uint32_t obs_len, uint32_t world, uint32_t depth, uint32_t kmax) {
    if (!layout_ok(n, obs_len, n) || world == 0 || depth < 2 || depth > XCHG_MAX_DEPTH || kmax == 0 ||
        kmax > XCHG_MAX_BATCH)
        return 0;
    return (size_t)depth * world * kmax * PackLayout{n, obs_len, n}.words();
}

extern "C" int cf2_xchg_register(cf2_xchg* x, uint32_t n, uint32_t obs_len, uint32_t watch_age, uint32_t kmax,
                                 float* const* obs_dev, uint8_t* const* reset_dev, uint32_t* send_dev,
                                 uint32_t* recv_dev, uint16_t* age_dev, uint32_t* overflow_dev, uint32_t* pred_dev,
                                 uint32_t npred) {
    // npred: a consume writes the rows of its steps and zeroes the CONSUME_MAX rows after them
    if (!x || x->registered || !obs_dev || !reset_dev || !send_dev || !recv_dev || !age_dev || kmax == 0 ||
        kmax > XCHG_MAX_BATCH || !layout_ok(n, obs_len, n) || (uint64_t)x->world * n >= (1ull << 31) ||
        npred > XCHG_MAX_PRED || (watch_age != 0xFFFFFFFFu && (npred < 2 * CONSUME_MAX + 1 || !pred_dev)))
        return CF2_ERR_INVALID_ARG;
    if (((uintptr_t)send_dev & 15u) || ((uintptr_t)recv_dev & 15u)) return CF2_ERR_INVALID_ARG;
    for (uint32_t j = 0; j < x->depth; ++j) {
        if (!obs_dev[j] || !reset_dev[j] || ((uintptr_t)obs_dev[j] & 15u)) return CF2_ERR_INVALID_ARG;
        x->obs[j] = obs_dev[j]; x->done[j] = reset_dev[j];
    }
    x->n = n; x->ol = obs_len; x->watch = watch_age; x->kmax = kmax;
    x->wmax = PackLayout{n, obs_len, n}.words();
    x->npred = watch_age != 0xFFFFFFFFu ? npred : 0u;
    x->pred = watch_age != 0xFFFFFFFFu ? pred_dev : nullptr;
    x->send = send_dev; x->recv = recv_dev;
    x->age = age_dev; x->overflow = overflow_dev;
    x->registered = true;
    return CF2_OK;
}

static uint32_t* xchg_send(const cf2_xchg* x, uint32_t q) { return x->send + (size_t)q * x->kmax * x->wmax; }
static uint32_t* xchg_recv(const cf2_xchg* x, uint32_t q) { return x->recv + (size_t)q * x->world * x->kmax * x->wmax; }
static uint32_t* xchg_scratch(const cf2_xchg* x, uint32_t q, uint32_t s) {
    return x->send + (size_t)x->depth * x->kmax * x->wmax + ((size_t)q * x->kmax + s) * PACK_SCRATCH_WORDS;
}

// the receivers' work of the nb steps k0 .. of one batch in region q (capacity cap), consume
// launches of up to CONSUME_MAX steps on the exchange stream
static int xchg_consume(cf2_xchg* x, uint64_t k0, uint32_t nb, uint32_t q, uint32_t cap, hipStream_t st_) {
    const PackLayout L{x->n, x->ol, cap};
    const uint32_t words = L.words();
    for (uint32_t s0 = 0; s0 < nb; s0 += CONSUME_MAX) {
        ConsumeSteps S;
        memset(&S, 0, sizeof(S));
        S.steps = nb - s0 < CONSUME_MAX ? nb - s0 : CONSUME_MAX;
        S.pk0 = xchg_recv(x, q) + (size_t)s0 * words;
        S.step_words = words;
        S.rank_stride = nb * words;                // the batch's [world][nb][words] layout
        if (x->pred) {
            S.ring = x->pred;
            S.npred = x->npred;
            S.row0 = (uint32_t)((k0 + s0) % x->npred);
            S.nzero = CONSUME_MAX;                 // the rows after the launch's last step
        }
        if (s0 == 0) {          // the batch's packs are done: zero its spill counters for the region's next use
            S.scratch = xchg_scratch(x, q, 0);
            S.scratch_words = nb * PACK_SCRATCH_WORDS;
        }
        const int st = consume_launch(S, x->world, L, x->age, x->overflow, x->watch, st_);
        if (st != CF2_OK) return st;
    }
    return CF2_OK;
}

// the look-ahead count ring to a host buffer on stream st, and the buffer's copy event (recorded
// after it)
static int xchg_copy_counts(cf2_xchg* x, uint32_t* pred_host, hipStream_t st_) {
    uint32_t slot = 0;
    while (slot < x->ncopy && x->copy_host[slot] != pred_host) ++slot;
    if (slot == x->ncopy) {
        if (x->ncopy == XCHG_MAX_COPIES) return CF2_ERR_INVALID_ARG;     // more host buffers than slots
        const hipError_t e = hipEventCreateWithFlags(&x->copy_ev[slot], hipEventDisableTiming);
        if (e != hipSuccess) return hip_fail(e);
        x->copy_host[slot] = pred_host;
        ++x->ncopy;
    }
    const int st = words_to_host(x->pred, pred_host, x->npred * x->world, st_);
    if (st != CF2_OK) return st;
    const hipError_t e = hipEventRecord(x->copy_ev[slot], st_);
    if (e != hipSuccess) return hip_fail(e);
    if (st_ == x->xs) x->last = x->copy_ev[slot];
    return CF2_OK;
}

// Inline exchanges (cf2_xchg_env_step, cf2_xchg_publish) run on the caller's stream and record no
// event; the library remembers that stream.  A caller on another stream (a region take, a wait)
// is ordered after it through one event recorded then, on the remembered stream.
static int xchg_after_inline(cf2_xchg* x, hipStream_t stream) {
    if (!x->inl || x->inl_stream == stream) return CF2_OK;
    hipError_t e = hipEventRecord(x->inl_ev, x->inl_stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(stream, x->inl_ev, 0);
    if (e != hipSuccess) return hip_fail(e);
    x->inl = false;           // everything inline so far is ordered before `stream` from now on
    return CF2_OK;
}

// The exchange of region q's batch (nb packed buffers at cap) after the env stream's work so far:
// the all-gather, the receivers' work and the look-ahead ring to pred_host (optional).  Batched
// (inl false): on the exchange stream, forked from the env stream, closed by region q's free event,
// so the next batch's env-steps overlap it.  Inline: on the env stream itself, for a consumer that
// needs every step's rows before it issues the next step (nothing to overlap): no fork, no event
// (each HIP event record or stream wait costs 2-6 us of host time; the eager step is host-bound).
static int xchg_exchange(cf2_xchg* x, uint64_t k0, uint32_t nb, uint32_t q, uint32_t cap, hipStream_t es,
                         uint32_t* pred_host, bool inl) {
    hipError_t e = hipSuccess;
    const hipStream_t xs = inl ? es : x->xs;
    if (!inl) {
        HostClock hc(x, 3);
        e = hipEventRecord(x->fork, es);
        if (e == hipSuccess) e = hipStreamWaitEvent(x->xs, x->fork, 0);
    }
    if (e != hipSuccess) return hip_fail(e);
    const size_t words = PackLayout{x->n, x->ol, cap}.words();
    {
        HostClock hc(x, 4);
        if (g_rccl.all_gather(xchg_send(x, q), xchg_recv(x, q), nb * words, ncclUint32, x->comm, xs) != ncclSuccess)
            return CF2_ERR_HIP;
    }
    int st;
    {
        HostClock hc(x, 5);
        st = xchg_consume(x, k0, nb, q, cap, xs);
    }
    if (st != CF2_OK) return st;
    HostClock hc(x, 6);
    if (inl) {
        x->free_rec[q] = false;          // its readers are ordered on es (xchg_after_inline for others)
        x->inl = true;
        x->inl_stream = es;
    } else {
        e = hipEventRecord(x->free_[q], x->xs);     // the region's buffers are read and its counters zeroed
        if (e != hipSuccess) return hip_fail(e);
        x->free_rec[q] = true;
        x->last = x->free_[q];       // one event closes a batch without a count copy
        x->end_rec = true;
    }
    if (pred_host && x->pred) {
        st = xchg_copy_counts(x, pred_host, xs);
        if (st != CF2_OK) return st;
    }
    return CF2_OK;
}

static int xchg_take_region(cf2_xchg* x, uint32_t region, hipStream_t es) {
    if (region != x->next_region % x->depth) return CF2_ERR_INVALID_ARG;     // the caller lost count
    int st = xchg_after_inline(x, es);
    if (st != CF2_OK) return st;
    ++x->next_region;
    if (!x->free_rec[region]) return CF2_OK;
    const hipError_t e = hipStreamWaitEvent(es, x->free_[region], 0);     // the all-gather that last read it
    return e == hipSuccess ? CF2_OK : hip_fail(e);
}

extern "C" int cf2_xchg_publish(cf2_xchg* x, uint64_t k, uint32_t cap, uint32_t region, void* env_stream) {
    if (!x || !x->registered || x->open || !layout_ok(x->n, x->ol, cap) || region >= x->depth)
        return CF2_ERR_INVALID_ARG;
    if (region != x->next_region % x->depth) return CF2_ERR_INVALID_ARG;
    const hipStream_t es = (hipStream_t)env_stream;
    int st = xchg_after_inline(x, es);
    if (st != CF2_OK) return st;
    ++x->next_region;
    // the caller's env-step wrote obs / done of the region (after cf2_xchg_wait_free): pack it here
    st = cf2_obs_pack(x->obs[region], x->done[region], x->n, x->ol, cap, xchg_send(x, region),
                      xchg_scratch(x, region, 0), nullptr, es);
    if (st != CF2_OK) return st;
    return xchg_exchange(x, k, 1, region, cap, es, nullptr, /*inl=*/true);
}

extern "C" int cf2_xchg_wait_free(cf2_xchg* x, uint32_t region, void* stream) {
    if (!x || region >= x->depth) return CF2_ERR_INVALID_ARG;
    const int st = xchg_after_inline(x, (hipStream_t)stream);
    if (st != CF2_OK) return st;
    if (!x->free_rec[region]) return CF2_OK;
    const hipError_t e = hipStreamWaitEvent((hipStream_t)stream, x->free_[region], 0);
    return e == hipSuccess ? CF2_OK : hip_fail(e);
}

extern "C" int cf2_xchg_wait(cf2_xchg* x, void* stream) {
    if (!x) return CF2_ERR_INVALID_ARG;
    const int st = xchg_after_inline(x, (hipStream_t)stream);
    if (st != CF2_OK) return st;
    if (!x->end_rec) return CF2_OK;
    const hipError_t e = hipStreamWaitEvent((hipStream_t)stream, x->last, 0);
    return e == hipSuccess ? CF2_OK : hip_fail(e);
}

extern "C" int cf2_xchg_pred_to_host(cf2_xchg* x, uint32_t* pred_host, void* stream) {
    if (!x || !x->registered || !x->pred || !pred_host) return CF2_ERR_INVALID_ARG;
    const hipStream_t st = (hipStream_t)stream;
    const int s2 = xchg_after_inline(x, st);
    if (s2 != CF2_OK) return s2;
    if (x->end_rec) {
        const hipError_t e = hipStreamWaitEvent(st, x->last, 0);
        if (e != hipSuccess) return hip_fail(e);
    }
    return words_to_host(x->pred, pred_host, x->npred * x->world, st);
}

// The host waits until the latest count copy into pred_host (cf2_xchg_run / cf2_xchg_end with that
// buffer) is complete.  CF2_ERR_INVALID_ARG if no exchange ever copied into it.
extern "C" int cf2_xchg_copy_sync(cf2_xchg* x, const uint32_t* pred_host) {
    if (!x || !pred_host) return CF2_ERR_INVALID_ARG;
    for (uint32_t k = 0; k < x->ncopy; ++k)
        if (x->copy_host[k] == pred_host) {
            const hipError_t e = hipEventSynchronize(x->copy_ev[k]);
            return e == hipSuccess ? CF2_OK : hip_fail(e);
        }
    return CF2_ERR_INVALID_ARG;
}

extern "C" int cf2_xchg_begin(cf2_xchg* x, uint32_t cap, uint32_t region, void* env_stream) {
    if (!x || !x->registered || x->open || region >= x->depth || !layout_ok(x->n, x->ol, cap))
        return CF2_ERR_INVALID_ARG;
    HostClock hc(x, 1);
    const int st = xchg_take_region(x, region, (hipStream_t)env_stream);
    if (st != CF2_OK) return st;
    x->open = true;
    x->open_region = region; x->open_cap = cap; x->open_steps = 0;
    return CF2_OK;
}

extern "C" int cf2_xchg_step(cf2_xchg* x, cf2_ctx* ctx, const float* act_dev, float* rew_dev, uint8_t* trunc_dev,
                             float* cost_dev, float* level_dev, void* env_stream) {
    if (!x || !x->open || !ctx || !act_dev || ((uintptr_t)act_dev & 15u) || !rew_dev || x->open_steps >= x->kmax)
        return CF2_ERR_INVALID_ARG;
    cf2_layout lay;      // the env-step writes n rows of obs_len into the registered buffers: they must match
    if (cf2_layout_get(ctx, &lay) != CF2_OK || lay.num_envs != x->n || lay.obs_len != x->ol) return CF2_ERR_INVALID_ARG;
    const hipStream_t es = (hipStream_t)env_stream;
    const uint32_t q = x->open_region, s = x->open_steps, cap = x->open_cap;
    uint32_t* pk = xchg_send(x, q) + (size_t)s * PackLayout{x->n, x->ol, cap}.words();
    uint32_t* scr = xchg_scratch(x, q, s);
    HostClock hc(x, 2);
    int st = cf2_step_packed(ctx, act_dev, x->obs[q], rew_dev, x->done[q], trunc_dev, cost_dev, level_dev, pk, scr,
                             cap, es);
    if (st == CF2_ERR_UNSUPPORTED) {      // a shape without the fused pack: the env-step, then the pack
        st = cf2_step(ctx, act_dev, nullptr, x->obs[q], rew_dev, x->done[q], trunc_dev, cost_dev, level_dev, nullptr,
                      es);
        if (st == CF2_OK) st = cf2_obs_pack(x->obs[q], x->done[q], x->n, x->ol, cap, pk, scr, nullptr, es);
    }
    if (st == CF2_OK) ++x->open_steps;
    return st;
}

extern "C" int cf2_xchg_end(cf2_xchg* x, uint64_t k0, uint32_t* pred_host, void* env_stream) {
    if (!x || !x->open || x->open_steps == 0) return CF2_ERR_INVALID_ARG;
    x->open = false;
    return xchg_exchange(x, k0, x->open_steps, x->open_region, x->open_cap, (hipStream_t)env_stream, pred_host,
                         /*inl=*/false);
}

static int xchg_run(cf2_xchg* x, cf2_ctx* ctx, uint64_t k0, uint32_t nb, uint32_t cap, uint32_t region,
                    const float* const* act_dev, uint32_t nact, float* rew_dev, uint8_t* trunc_dev, float* cost_dev,
                    float* level_dev, uint32_t* pred_host, void* env_stream, bool inl) {
    if (!x || !x->registered || x->open || !ctx || !act_dev || nact == 0 || nb == 0 || nb > x->kmax ||
        region >= x->depth || !layout_ok(x->n, x->ol, cap) || !rew_dev)
        return CF2_ERR_INVALID_ARG;
    for (uint32_t a = 0; a < nact; ++a)
        if (!act_dev[a] || ((uintptr_t)act_dev[a] & 15u)) return CF2_ERR_INVALID_ARG;
    HostClock hc(x, 0);
    if (x->timing) ++x->host_calls;
    int st = cf2_xchg_begin(x, cap, region, env_stream);
    if (st != CF2_OK) return st;           // nothing taken
    for (uint32_t s = 0; st == CF2_OK && s < nb; ++s)
        st = cf2_xchg_step(x, ctx, act_dev[(k0 + s) % nact], rew_dev, trunc_dev, cost_dev, level_dev, env_stream);
    if (st != CF2_OK) {
        // the batch is abandoned: the region is given back (the caller's count, which a failed call
        // does not advance, stays in step with ours) and the spill counters its packs took so far
        // are zeroed, so the region's next use starts from empty counters as after an exchange
        x->open = false;
        --x->next_region;
        if (x->open_steps > 0)
            (void)hipMemsetAsync(xchg_scratch(x, region, 0), 0, (size_t)x->open_steps * PACK_SCRATCH_WORDS * sizeof(uint32_t),
                                 (hipStream_t)env_stream);
        return st;
    }
    if (!inl) return cf2_xchg_end(x, k0, pred_host, env_stream);
    x->open = false;
    return xchg_exchange(x, k0, x->open_steps, x->open_region, x->open_cap, (hipStream_t)env_stream, pred_host,
                         /*inl=*/true);
}

extern "C" int cf2_xchg_run(cf2_xchg* x, cf2_ctx* ctx, uint64_t k0, uint32_t nb, uint32_t cap, uint32_t region,
                            const float* const* act_dev, uint32_t nact, float* rew_dev, uint8_t* trunc_dev,
                            float* cost_dev, float* level_dev, uint32_t* pred_host, void* env_stream) {
    return xchg_run(x, ctx, k0, nb, cap, region, act_dev, nact, rew_dev, trunc_dev, cost_dev, level_dev, pred_host,
                    env_stream, /*inl=*/false);
}

// One env-step and its exchange, all on env_stream (inline: for a consumer that needs each step's
// gathered rows before it issues the next step, so there is nothing to overlap); pred_host, if
// given, receives the look-ahead counts (cf2_xchg_copy_sync)
extern "C" int cf2_xchg_env_step(cf2_xchg* x, cf2_ctx* ctx, uint64_t k, uint32_t cap, uint32_t region,
                                 const float* act_dev, float* rew_dev, uint8_t* trunc_dev, float* cost_dev,
                                 float* level_dev, uint32_t* pred_host, void* env_stream) {
    return xchg_run(x, ctx, k, 1, cap, region, &act_dev, 1, rew_dev, trunc_dev, cost_dev, level_dev, pred_host,
                    env_stream, /*inl=*/true);
}

// Diagnostics: the host time of the exchange's C calls by part (XCHG_HOST_PARTS ns sums, see the
// constant's comment) and the number of cf2_xchg_run / env_step calls they cover; all zero unless
// CF2_XCHG_HOST_TIMING=1 was set when the exchange was created.  reset != 0 clears them.
extern "C" int cf2_xchg_host_times(cf2_xchg* x, double* ns_out, uint32_t n_out, uint64_t* calls_out, int reset) {
    if (!x || !ns_out || n_out < (uint32_t)XCHG_HOST_PARTS || !calls_out) return CF2_ERR_INVALID_ARG;
    for (int p = 0; p < XCHG_HOST_PARTS; ++p) ns_out[p] = x->host_ns[p];
    *calls_out = x->host_calls;
    if (reset) {
        for (int p = 0; p < XCHG_HOST_PARTS; ++p) x->host_ns[p] = 0.0;
        x->host_calls = 0;
    }
    return CF2_OK;
}
