// cf2sim_pack.h -- the packed buffer of the delta observation exchange,
// shared by the standalone pack kernel (cf2sim_exchange.hip) and the env-step kernel's fused pack
// epilogue (cf2sim_kernels.hip, step_kernel_small).
//
// One rank's packed buffer (32-bit words, 16-B multiple):
//   [0] 0 (reserved)   [1] n   [2] OL   [3] cap     (informational: no receiver reads them; the
//                                                    env-step's fused pack does not write them)
//   [4, 4 + n OL)                       o_k rows
//   [.., + ceil(n / 32))                reset bitmap, env i = bit i % 32 of word i / 32
//   [.., + ceil(n / 64))                block table: per 64-env pack block, the first spill slot of its
//                                       resets past its quota (or PACK_DROPPED: the spill area had no
//                                       room for them; 0 when the block has no more than its quota)
//   [.., + cap (OL + 5))                side entries: local env index, o_0[OL], A[4]
// Side slots: the first nblk * quota slots belong to the pack blocks, quota consecutive slots each,
// taken by the block's first quota resets in env order with no atomic; the rest of the capacity is
// a shared spill area, where a block with more resets than its quota takes the excess as
// consecutive slots with one atomic on a counter.  quota = min(cap, default crash budget) / nblk
// (at most 64), the default budget being 7.5 % of the shard (cf2sim.dist.default_cap): at it the
// quota is 4 and 88 % of the blocks of the steady 4.1 % reset rate need no atomic.  Capacity above
// the budget (the predicted time-outs the caller adds) all goes to the spill area, so predicted
// time-outs fit however they fall over the blocks.  (With quota = cap / nblk, a capacity just above
// a multiple of nblk -- 2575 at 32 768 envs -- left a spill area of 15 slots: quota 5 instead of 4
// and overflows at a reset count half the capacity, tools/xchg_watch_probe.py, gpurun_out/r06b.)  Every block
// taking its slots from one counter serialised at the memory-side atomic unit (~35 ns per atomic on
// one address: 19.5 us for a 32 768-env pack, round 4); eight per-XCD counters (round 5) still cost
// the fused step ~2 us at 32 768 envs.
// The counter lives in a per-buffer scratch area that is never sent (PACK_SCRATCH_WORDS after the
// largest packed buffer).  The standalone pack zeroes the scratch of the buffer the next pack on its
// stream uses; cf2_xchg_* zeroes a batch's counters in its consume, once the batch's packs are done.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cf2 {

constexpr uint32_t XB_PACK = 64;                  // envs per pack block (one block-table word each)
constexpr uint32_t PACK_DROPPED = 0xFFFFFFFFu;     // block-table value: its resets past the quota got no slot
constexpr uint32_t PACK_SCRATCH_WORDS = 32;     // the spill counter (one 128-B line)

struct PackLayout {
    uint32_t n, ol, cap;
    __host__ __device__ uint32_t od() const { return 2u * (ol + 4u); }
    __host__ __device__ uint32_t o_slab() const { return 4u; }
    __host__ __device__ uint32_t bits() const { return 4u + n * ol; }
    __host__ __device__ uint32_t btab() const { return bits() + (n + 31u) / 32u; }
    __host__ __device__ uint32_t side() const { return btab() + (n + XB_PACK - 1u) / XB_PACK; }
    __host__ __device__ uint32_t entry() const { return ol + 5u; }
    __host__ __device__ uint32_t words() const { return (side() + cap * entry() + 3u) & ~3u; }
    __host__ __device__ uint32_t nblk() const { return (n + XB_PACK - 1u) / XB_PACK; }
    // the default crash budget of an n-env shard: 7.5 %, at least 64, at most n (dist.default_cap)
    __host__ __device__ uint32_t budget() const {
        const uint32_t c = (3u * n + 39u) / 40u;
        return c < 64u ? (n < 64u ? n : 64u) : (c < n ? c : n);
    }
    // side slots each pack block owns, then the start and size of the shared spill area
    __host__ __device__ uint32_t quota() const {
        const uint32_t c = cap < budget() ? cap : budget(), q = c / nblk();
        return q < XB_PACK ? q : XB_PACK;
    }
    __host__ __device__ uint32_t spill_base() const { return nblk() * quota(); }
    __host__ __device__ uint32_t spill() const { return cap - spill_base(); }
};

// The exchange's pack fused into the env-step (cf2_step_packed): where step_kernel_small writes the
// packed buffer of its envs besides their observation rows
struct PackIO {
    uint32_t* pk;              // packed buffer (null: no pack)
    uint32_t* scratch;         // this buffer's spill counter (zeroed before the env-step)
    uint32_t cap;
};

// The block-table word of a pack block with c resets (one thread calls it): 0 when they fit the
// block's quota, else the first of c - quota consecutive spill slots, or PACK_DROPPED when the spill
// area has no room for them (a failed attempt leaves the counter past the area, so it overflows
// only within one block's excess of full).
__device__ __forceinline__ uint32_t pack_alloc(const PackLayout& L, uint32_t* scratch, uint32_t c) {
    const uint32_t q = L.quota();
    if (c <= q) return 0u;
    const uint32_t e = c - q, old = atomicAdd(scratch, e);
    return old + e <= L.spill() ? L.spill_base() + old : PACK_DROPPED;
}

// The side slot of the reset of rank `rank` (resets before it in its pack block) in block blk, whose
// block-table word is `first`, or PACK_DROPPED
__host__ __device__ __forceinline__ uint32_t pack_entry_slot(const PackLayout& L, uint32_t blk, uint32_t rank,
                                                             uint32_t first) {
    const uint32_t q = L.quota();
    if (rank < q) return blk * q + rank;
    return first == PACK_DROPPED ? PACK_DROPPED : first + (rank - q);
}

// The side slot of local env li (a reset env) from the block table and the bitmap, or PACK_DROPPED.
__device__ __forceinline__ uint32_t pack_slot(const uint32_t* pk, const PackLayout& L, uint32_t li) {
    const uint32_t b = li / XB_PACK, w0 = b * (XB_PACK / 32u), wl = li / 32u;
    uint32_t rank = 0;
    for (uint32_t w = w0; w < wl; ++w) rank += (uint32_t)__popc(pk[L.bits() + w]);
    rank += (uint32_t)__popc(pk[L.bits() + wl] & ((1u << (li % 32u)) - 1u));
    return pack_entry_slot(L, b, rank, pk[L.btab() + b]);
}

}  // namespace cf2
