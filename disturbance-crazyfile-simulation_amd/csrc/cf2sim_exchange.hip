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
// and every receiver rebuilds the full [N_total, OD] slab from its previous one.  The action slots
// follow the reference's history aliasing (compute_history with the action deque holding the
// action buffer's last entry right after a reset, envs/base.py:455-462; the kernel's halias flags):
// with `age` = env-steps since the env's last reset (0 = reset this step; uint16, saturating),
//   age 1:  A0 = A1 = a_k           (both history slots alias the action buffer, which after the
//                                     step holds a_k in every row: aggregate_phy_steps is a
//                                     multiple of buf_size, as in the reference's default env)
//   age 2:  A0 = a_k, A1 = a_{k-1}
//   age 3+: A0 = the previous row's A1, A1 = a_{k-1}
// where a_k is the action of the env-step that produced the row.  The receiver tracks age from the
// bitmaps (exact: reset or not is always known).  More resets than `cap` on a rank in one step
// (an overflow) leaves those rows' o_0 / A parts unknown: the receiver writes NaN there and counts
// the overflow; the rows of the following steps are exact again.
// The capacity may change from step to step (the caller sizes the all-gather): TimeLimit
// truncations are predictable, so the receiver counts, per rank, the envs whose age reaches
// max_steps - L this step -- at most that many time out L steps later (fewer if they crash first)
// -- into pred[step % (L + 1)][rank], and the caller adds that count to the crash budget of step
// + L.  Every rank holds the same ages, so every rank derives the same capacity.
//
// Packed buffer of one rank (32-bit words, 16-B multiple; cf2_obs_packed_words):
//   [0] reset count (may exceed cap)   [1] n   [2] OL   [3] cap
//   [4, 4 + n OL)                       o_k rows
//   [.., + ceil(n / 32))                reset bitmap, env i = bit i % 32 of word i / 32
//   [.., + ceil(n / 256))               block table: the first side slot of each 256-env pack block
//                                       (a block's resets hold consecutive slots, in env order)
//   [.., + cap (OL + 5))                side entries: local env index, o_0[OL], A[4]
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <dlfcn.h>
#include <stdint.h>
#include <string.h>
#include <math.h>
#include <mutex>
#include "../../include/cf2sim.h"
#include "cf2sim_internal.h"

namespace cf2 {

constexpr uint32_t XB_PACK = 256;   // envs per pack block (one block-table word each)

struct PackLayout {
    uint32_t n, ol, cap;
    __host__ __device__ uint32_t od() const { return 2u * (ol + 4u); }
    __host__ __device__ uint32_t o_slab() const { return 4u; }
    __host__ __device__ uint32_t bits() const { return 4u + n * ol; }
    __host__ __device__ uint32_t btab() const { return bits() + (n + 31u) / 32u; }
    __host__ __device__ uint32_t side() const { return btab() + (n + XB_PACK - 1u) / XB_PACK; }
    __host__ __device__ uint32_t entry() const { return ol + 5u; }
    __host__ __device__ uint32_t words() const { return (side() + cap * entry() + 3u) & ~3u; }
};

constexpr uint32_t XB = XB_PACK;    // rows per block

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
// run of the o_k slab; the reset bitmap comes from wave ballots; the block's resets take
// consecutive side slots from one atomic per block on the count word (per-wave atomics on that one
// word serialised at the L2: 19.5 us per 32 768-env pack), in an order that is immaterial (each
// entry carries its env index).  clear_next: the count word of the buffer the next pack on this
// stream writes (its previous contents were gathered already), so the counts need no memset.
template <uint32_t OL>
__global__ void __launch_bounds__(XB) obs_pack_kernel(const float* __restrict__ obs, const uint8_t* __restrict__ reset,
                                                      PackLayout L, uint32_t* __restrict__ pk,
                                                      uint32_t* __restrict__ clear_next) {
    constexpr uint32_t OD = 2u * (OL + 4u);
    __shared__ __align__(16) float s_rows[XB * OD];
    __shared__ __align__(16) float s_o[XB * OL];
    __shared__ uint32_t s_wcnt[XB / 64u + 1u];
    const uint32_t tid = threadIdx.x, base = blockIdx.x * XB, i = base + tid, lane = tid & 63u, wv = tid >> 6;
    const uint32_t nrow = L.n - base < XB ? L.n - base : XB;
    if (blockIdx.x == 0 && tid == 0) {
        if (clear_next) clear_next[0] = 0u;
        pk[1] = L.n; pk[2] = OL; pk[3] = L.cap;
    }
    const bool live = tid < nrow;
    const bool r = live && reset[i] != 0;
    const uint64_t m = __ballot(r);
    if (lane == 0) s_wcnt[wv] = (uint32_t)__popcll(m);
    rows_to_lds(s_rows, obs + (size_t)base * OD, nrow * OD, ((uintptr_t)obs & 15u) == 0 && (base * OD) % 4u == 0);
    __syncthreads();
    const float* row = s_rows + tid * OD;
    if (live) {
#pragma unroll
        for (uint32_t k = 0; k < OL; ++k) s_o[tid * OL + k] = row[OL + 4u + k];
    }
    uint32_t* bits = pk + L.bits();
    const uint32_t wbase = base + (tid & ~63u);
    if (lane == 0 && wbase < L.n) bits[wbase / 32u] = (uint32_t)m;
    if (lane == 32 && wbase + 32u < L.n) bits[wbase / 32u + 1u] = (uint32_t)(m >> 32);
    if (tid == 0) {
        uint32_t tot = 0;
#pragma unroll
        for (uint32_t w = 0; w < XB / 64u; ++w) { const uint32_t c = s_wcnt[w]; s_wcnt[w] = tot; tot += c; }
        const uint32_t first = tot ? atomicAdd(pk, tot) : 0u;     // the block's first side slot
        s_wcnt[XB / 64u] = first;
        pk[L.btab() + blockIdx.x] = first;
    }
    __syncthreads();
    if (r) {
        const uint32_t slot = s_wcnt[XB / 64u] + s_wcnt[wv] + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (slot < L.cap) {
            uint32_t* e = pk + L.side() + slot * L.entry();
            e[0] = i;
            float* ef = reinterpret_cast<float*>(e + 1);
#pragma unroll
            for (uint32_t k = 0; k < OL + 4u; ++k) ef[k] = row[k];     // o_0 and A (= A_0)
        }
    }
    lds_to_rows(reinterpret_cast<float*>(pk + L.o_slab()) + (size_t)base * OL, s_o, nrow * OL,
                ((uintptr_t)pk & 15u) == 0 && (base * OL) % 4u == 0);
}

// Receiver: one thread per global env (rank r = i / n).  The block's previous rows are read
// coalesced into LDS, each thread rebuilds its row there (a reset row from its side entry, found
// through the block table and the bitmap; NaN in its o_0 / A parts if the env's rank overflowed its
// side slab), the block writes them out coalesced.  One launch (the reset entries used to take a
// second, scattered-write kernel: 5.6 us on 262 144 rows).
template <uint32_t OL>
__global__ void __launch_bounds__(XB) obs_unpack_rows_kernel(const uint32_t* __restrict__ pk_all, uint32_t words,
                                                             uint32_t world, PackLayout L,
                                                             const float* __restrict__ act,
                                                             const float* __restrict__ act_prev,
                                                             uint16_t* __restrict__ age,
                                                             const float* __restrict__ slab_prev,
                                                             float* __restrict__ slab, uint32_t* __restrict__ overflow,
                                                             uint32_t watch_age, uint32_t* __restrict__ pred,
                                                             uint32_t* __restrict__ pred_next) {
    constexpr uint32_t OD = 2u * (OL + 4u);
    __shared__ __align__(16) float s_rows[XB * OD];
    const uint32_t tid = threadIdx.x, base = blockIdx.x * XB, i = base + tid;
    const uint32_t total = world * L.n;
    const uint32_t nrow = total - base < XB ? total - base : XB;
    const bool al = (base * OD) % 4u == 0 && ((uintptr_t)slab_prev & 15u) == 0 && ((uintptr_t)slab & 15u) == 0;
    if (blockIdx.x == 0 && pred_next && tid < world) pred_next[tid] = 0u;     // the next step's counts
    // this thread's inputs first (their latency overlaps the block's row copy)
    const bool live = tid < nrow;
    const uint32_t ic = live ? i : total - 1u;
    const uint32_t r = ic / L.n, li = ic - r * L.n;
    const uint32_t* pk = pk_all + (size_t)r * words;
    const float* okp = reinterpret_cast<const float*>(pk + L.o_slab()) + (size_t)li * OL;
    float ok[OL];
#pragma unroll
    for (uint32_t k = 0; k < OL; ++k) ok[k] = okp[k];
    const bool rs = (pk[L.bits() + li / 32u] >> (li % 32u)) & 1u;
    const uint32_t a_old = age[ic];
    const float4 ak = reinterpret_cast<const float4*>(act)[ic];
    const float4 ap = reinterpret_cast<const float4*>(act_prev)[ic];
    const bool ovf = pk[0] > L.cap;
    rows_to_lds(s_rows, slab_prev + (size_t)base * OD, nrow * OD, al);
    __syncthreads();
    uint32_t a_new = 0xFFFFFFFFu;
    if (live) {
        float* row = s_rows + tid * OD;
        if (rs) {
#pragma unroll
            for (uint32_t k = 0; k < OL; ++k) row[OL + 4u + k] = ok[k];
            // the reset's side entry: the pack block's first slot plus the resets before this env in
            // its block (a block's slots are consecutive and in env order)
            const uint32_t pb = li / XB_PACK, wl = li / 32u;
            uint32_t slot = pk[L.btab() + pb];
            for (uint32_t w = pb * (XB_PACK / 32u); w < wl; ++w) slot += (uint32_t)__popc(pk[L.bits() + w]);
            slot += (uint32_t)__popc(pk[L.bits() + wl] & ((1u << (li % 32u)) - 1u));
            if (ovf || slot >= L.cap) {     // o_0 and A were not sent: marked unknown
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
            age[i] = 0;
            a_new = 0;
        } else {
            const uint32_t a = a_old < 0xFFFFu ? a_old + 1u : 0xFFFFu;
            const float akv[4] = {ak.x, ak.y, ak.z, ak.w}, apv[4] = {ap.x, ap.y, ap.z, ap.w};
            float a0[4], a1[4];
#pragma unroll
            for (uint32_t k = 0; k < 4u; ++k) {
                a0[k] = a >= 3u ? row[2u * OL + 4u + k] : akv[k];
                a1[k] = a == 1u ? akv[k] : apv[k];
            }
#pragma unroll
            for (uint32_t k = 0; k < OL; ++k) row[k] = row[OL + 4u + k];
#pragma unroll
            for (uint32_t k = 0; k < 4u; ++k) row[OL + k] = a0[k];
#pragma unroll
            for (uint32_t k = 0; k < OL; ++k) row[OL + 4u + k] = ok[k];
#pragma unroll
            for (uint32_t k = 0; k < 4u; ++k) row[2u * OL + 4u + k] = a1[k];
            age[i] = (uint16_t)a;
            a_new = a;
        }
    }
    // time-out look-ahead: envs at age watch_age time out (unless they crash first) L steps later
    if (pred && a_new == watch_age) atomicAdd(pred + r, 1u);     // ~1/max_steps of the envs per step
    if (overflow && live && li == 0 && ovf) atomicAdd(overflow, 1u);   // one count per overflowing rank
    __syncthreads();
    lds_to_rows(slab + (size_t)base * OD, s_rows, nrow * OD, al);
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
                            uint32_t* packed_dev, uint32_t* clear_next_dev, void* stream) {
    if (!obs_dev || !reset_dev || !packed_dev || !layout_ok(n, obs_len, cap)) return CF2_ERR_INVALID_ARG;
    if (((uintptr_t)obs_dev & 7u) || ((uintptr_t)packed_dev & 15u)) return CF2_ERR_INVALID_ARG;
    const PackLayout L{n, obs_len, cap};
    if (obs_len == 13u)
        hipLaunchKernelGGL(obs_pack_kernel<13>, dim3((n + XB - 1) / XB), dim3(XB), 0, (hipStream_t)stream, obs_dev,
                           reset_dev, L, packed_dev, clear_next_dev);
    else
        hipLaunchKernelGGL(obs_pack_kernel<17>, dim3((n + XB - 1) / XB), dim3(XB), 0, (hipStream_t)stream, obs_dev,
                           reset_dev, L, packed_dev, clear_next_dev);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? CF2_OK : hip_fail(e);
}

extern "C" int cf2_obs_unpack(const uint32_t* packed_all_dev, uint32_t world, uint32_t n, uint32_t obs_len,
                              uint32_t cap, const float* act_dev, const float* act_prev_dev, uint16_t* age_dev,
                              const float* slab_prev_dev, float* slab_dev, uint32_t* overflow_dev, uint32_t watch_age,
                              uint32_t* pred_dev, uint32_t* pred_next_dev, void* stream) {
    if (!packed_all_dev || !act_dev || !act_prev_dev || !age_dev || !slab_prev_dev || !slab_dev || world == 0 ||
        !layout_ok(n, obs_len, cap) || (uint64_t)world * n >= (1ull << 31))
        return CF2_ERR_INVALID_ARG;
    if (slab_prev_dev == slab_dev) return CF2_ERR_INVALID_ARG;     // rows are rebuilt from the previous slab
    if (((uintptr_t)act_dev & 15u) || ((uintptr_t)act_prev_dev & 15u) || ((uintptr_t)packed_all_dev & 15u) ||
        ((uintptr_t)slab_dev & 7u) || ((uintptr_t)slab_prev_dev & 7u))
        return CF2_ERR_INVALID_ARG;
    const PackLayout L{n, obs_len, cap};
    const uint32_t words = L.words(), total = world * n;
    if (obs_len == 13u)
        hipLaunchKernelGGL(obs_unpack_rows_kernel<13>, dim3((total + XB - 1) / XB), dim3(XB), 0, (hipStream_t)stream,
                           packed_all_dev, words, world, L, act_dev, act_prev_dev, age_dev, slab_prev_dev, slab_dev,
                           overflow_dev, watch_age, pred_dev, pred_next_dev);
    else
        hipLaunchKernelGGL(obs_unpack_rows_kernel<17>, dim3((total + XB - 1) / XB), dim3(XB), 0, (hipStream_t)stream,
                           packed_all_dev, words, world, L, act_dev, act_prev_dev, age_dev, slab_prev_dev, slab_dev,
                           overflow_dev, watch_age, pred_dev, pred_next_dev);
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
constexpr uint32_t XCHG_MAX_DEPTH = 8;
}  // namespace

constexpr uint32_t XCHG_MAX_PRED = 64, XCHG_MAX_PRED_EV = 16;

struct cf2_xchg {
    ncclComm_t comm;
    uint32_t world, rank, depth;
    hipEvent_t fork;
    hipEvent_t end[XCHG_MAX_DEPTH];
    bool pending[XCHG_MAX_DEPTH];      // slot's exchange issued: the next env-step into it waits for end[slot]
    bool recorded[XCHG_MAX_DEPTH];     // end[slot] has been recorded at least once
    // registered buffers (cf2_xchg_register) for cf2_xchg_env_step
    bool registered;
    uint32_t n, ol, watch, npred;
    float* obs[XCHG_MAX_DEPTH];
    uint8_t* done[XCHG_MAX_DEPTH];
    uint32_t* send[XCHG_MAX_DEPTH];
    uint32_t* recv[XCHG_MAX_DEPTH];
    float* slab[2];
    uint16_t* age;
    uint32_t* overflow;
    uint32_t* pred[XCHG_MAX_PRED];
    // the look-ahead ring copied to pinned host memory every pred_batch env-steps, each copy
    // followed by an event of a ring of npev (cf2_xchg_pred_sync)
    uint32_t* pred_host;
    uint32_t pred_batch, npev;
    hipEvent_t pev[XCHG_MAX_PRED_EV];
    hipStream_t comm_stream;
};

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

extern "C" int cf2_xchg_create(const uint8_t* id, size_t id_len, uint32_t world, uint32_t rank, uint32_t depth,
                               cf2_xchg** out) {
    if (!id || id_len < sizeof(ncclUniqueId) || !out || world == 0 || rank >= world || depth == 0 ||
        depth > XCHG_MAX_DEPTH)
        return CF2_ERR_INVALID_ARG;
    if (!g_rccl.init) return CF2_ERR_UNSUPPORTED;
    *out = nullptr;
    cf2_xchg* x = new cf2_xchg();
    x->world = world; x->rank = rank; x->depth = depth;
    hipError_t e = hipEventCreateWithFlags(&x->fork, hipEventDisableTiming);
    uint32_t made = 0;
    for (; e == hipSuccess && made < depth; ++made) e = hipEventCreateWithFlags(&x->end[made], hipEventDisableTiming);
    if (e != hipSuccess) {
        for (uint32_t k = 0; k + 1 < made; ++k) (void)hipEventDestroy(x->end[k]);
        if (made) (void)hipEventDestroy(x->fork);
        delete x;
        return hip_fail(e);
    }
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    if (g_rccl.init(&x->comm, (int)world, uid, (int)rank) != ncclSuccess) {
        for (uint32_t k = 0; k < depth; ++k) (void)hipEventDestroy(x->end[k]);
        (void)hipEventDestroy(x->fork);
        delete x;
        return CF2_ERR_HIP;
    }
    *out = x;
    return CF2_OK;
}

extern "C" int cf2_xchg_destroy(cf2_xchg* x) {
    if (!x) return CF2_OK;
    int st = CF2_OK;
    for (uint32_t k = 0; k < x->npev; ++k) (void)hipEventDestroy(x->pev[k]);
    if (g_rccl.destroy && g_rccl.destroy(x->comm) != ncclSuccess) st = CF2_ERR_HIP;
    for (uint32_t k = 0; k < x->depth; ++k) (void)hipEventDestroy(x->end[k]);
    (void)hipEventDestroy(x->fork);
    delete x;
    return st;
}

extern "C" int cf2_xchg_step(cf2_xchg* x, uint32_t slot, const float* obs_dev, const uint8_t* reset_dev, uint32_t n,
                             uint32_t obs_len, uint32_t cap, uint32_t* send_dev, uint32_t* send_next_dev,
                             uint32_t* recv_dev, const float* act_dev, const float* act_prev_dev, uint16_t* age_dev,
                             const float* slab_prev_dev, float* slab_dev, uint32_t* overflow_dev, uint32_t watch_age,
                             uint32_t* pred_dev, uint32_t* pred_next_dev, void* env_stream, void* comm_stream) {
    if (!x || slot >= x->depth || !recv_dev || !layout_ok(n, obs_len, cap)) return CF2_ERR_INVALID_ARG;
    const hipStream_t cs = (hipStream_t)comm_stream;
    hipError_t e = hipEventRecord(x->fork, (hipStream_t)env_stream);     // the env-step that wrote obs / done
    if (e == hipSuccess) e = hipStreamWaitEvent(cs, x->fork, 0);
    if (e != hipSuccess) return hip_fail(e);
    int st = cf2_obs_pack(obs_dev, reset_dev, n, obs_len, cap, send_dev, send_next_dev, comm_stream);
    if (st != CF2_OK) return st;
    const size_t words = PackLayout{n, obs_len, cap}.words();
    if (g_rccl.all_gather(send_dev, recv_dev, words, ncclUint32, x->comm, cs) != ncclSuccess) return CF2_ERR_HIP;
    st = cf2_obs_unpack(recv_dev, x->world, n, obs_len, cap, act_dev, act_prev_dev, age_dev, slab_prev_dev, slab_dev,
                        overflow_dev, watch_age, pred_dev, pred_next_dev, comm_stream);
    if (st != CF2_OK) return st;
    e = hipEventRecord(x->end[slot], cs);
    if (e != hipSuccess) return hip_fail(e);
    x->pending[slot] = x->recorded[slot] = true;
    return CF2_OK;
}

extern "C" int cf2_xchg_wait(cf2_xchg* x, uint32_t slot, void* stream) {
    if (!x || slot >= x->depth) return CF2_ERR_INVALID_ARG;
    if (!x->recorded[slot]) return CF2_OK;
    const hipError_t e = hipStreamWaitEvent((hipStream_t)stream, x->end[slot], 0);
    return e == hipSuccess ? CF2_OK : hip_fail(e);
}

extern "C" int cf2_xchg_register(cf2_xchg* x, uint32_t n, uint32_t obs_len, uint32_t watch_age, float* const* obs_dev,
                                 uint8_t* const* reset_dev, uint32_t* const* send_dev, uint32_t* const* recv_dev,
                                 float* slab0_dev, float* slab1_dev, uint16_t* age_dev, uint32_t* overflow_dev,
                                 uint32_t* const* pred_dev, uint32_t npred, uint32_t* pred_host, uint32_t pred_batch,
                                 uint32_t pred_events, void* comm_stream) {
    if (!x || x->registered || !obs_dev || !reset_dev || !send_dev || !recv_dev || !slab0_dev || !slab1_dev ||
        !age_dev || !layout_ok(n, obs_len, n) || npred > XCHG_MAX_PRED || pred_events > XCHG_MAX_PRED_EV ||
        (watch_age != 0xFFFFFFFFu && (npred < 2 || !pred_dev)) ||
        (pred_host && (watch_age == 0xFFFFFFFFu || pred_batch == 0 || pred_events == 0)))
        return CF2_ERR_INVALID_ARG;
    for (uint32_t r = 1; r < npred; ++r)           // one [npred][world] array
        if (pred_dev[r] != pred_dev[0] + (size_t)r * x->world) return CF2_ERR_INVALID_ARG;
    if (pred_host) {
        hipError_t e = hipSuccess;
        for (; e == hipSuccess && x->npev < pred_events; ++x->npev)
            e = hipEventCreateWithFlags(&x->pev[x->npev], hipEventDisableTiming);
        if (e != hipSuccess) {
            --x->npev;
            for (uint32_t k = 0; k < x->npev; ++k) (void)hipEventDestroy(x->pev[k]);
            x->npev = 0;
            return hip_fail(e);
        }
    }
    x->pred_host = pred_host;
    x->pred_batch = pred_batch;
    for (uint32_t j = 0; j < x->depth; ++j) {
        if (!obs_dev[j] || !reset_dev[j] || !send_dev[j] || !recv_dev[j]) return CF2_ERR_INVALID_ARG;
        x->obs[j] = obs_dev[j]; x->done[j] = reset_dev[j]; x->send[j] = send_dev[j]; x->recv[j] = recv_dev[j];
    }
    for (uint32_t r = 0; r < npred; ++r) x->pred[r] = pred_dev[r];
    x->n = n; x->ol = obs_len; x->watch = watch_age; x->npred = npred;
    x->slab[0] = slab0_dev; x->slab[1] = slab1_dev;
    x->age = age_dev; x->overflow = overflow_dev;
    x->comm_stream = (hipStream_t)comm_stream;
    x->registered = true;
    return CF2_OK;
}

extern "C" int cf2_xchg_env_step(cf2_xchg* x, cf2_ctx* ctx, uint64_t k, uint32_t cap, const float* act_dev,
                                 const float* act_all_dev, const float* act_prev_all_dev, float* rew_dev,
                                 uint8_t* trunc_dev, float* cost_dev, float* level_dev, void* env_stream) {
    if (!x || !x->registered || !ctx) return CF2_ERR_INVALID_ARG;
    const uint32_t j = (uint32_t)(k % x->depth);
    const hipStream_t es = (hipStream_t)env_stream;
    if (x->pending[j]) {                 // the exchange that last read buffer j
        const hipError_t e = hipStreamWaitEvent(es, x->end[j], 0);
        if (e != hipSuccess) return hip_fail(e);
        x->pending[j] = false;
    }
    int st = cf2_step(ctx, act_dev, nullptr, x->obs[j], rew_dev, x->done[j], trunc_dev, cost_dev, level_dev, nullptr,
                      env_stream);
    if (st != CF2_OK) return st;
    const bool w = x->watch != 0xFFFFFFFFu;
    st = cf2_xchg_step(x, j, x->obs[j], x->done[j], x->n, x->ol, cap, x->send[j], x->send[(j + 1) % x->depth],
                       x->recv[j], act_all_dev, act_prev_all_dev, x->age, x->slab[(k + 1) % 2], x->slab[k % 2],
                       x->overflow, x->watch, w ? x->pred[k % x->npred] : nullptr,
                       w ? x->pred[(k + 1) % x->npred] : nullptr, env_stream, x->comm_stream);
    if (st != CF2_OK || !x->pred_host || k % x->pred_batch) return st;
    hipError_t e = hipMemcpyAsync(x->pred_host, x->pred[0], (size_t)x->npred * x->world * sizeof(uint32_t),
                                  hipMemcpyDeviceToHost, x->comm_stream);
    if (e == hipSuccess) e = hipEventRecord(x->pev[(k / x->pred_batch) % x->npev], x->comm_stream);
    return e == hipSuccess ? CF2_OK : hip_fail(e);
}

extern "C" int cf2_xchg_pred_sync(cf2_xchg* x, uint64_t k) {
    if (!x || !x->pred_host || k % x->pred_batch) return CF2_ERR_INVALID_ARG;
    const hipError_t e = hipEventSynchronize(x->pev[(k / x->pred_batch) % x->npev]);
    return e == hipSuccess ? CF2_OK : hip_fail(e);
}
