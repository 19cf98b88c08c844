// cf2sim_pack.h -- the packed buffer of the delta observation exchange,
// shared by the standalone pack kernel (cf2sim_exchange.hip) and the env-step kernel's fused pack
// epilogue (cf2sim_kernels.hip, step_kernel_small).
//
// One rank's packed buffer (32-bit words, 16-B multiple):
//   [0] 0 (reserved)   [1] n   [2] OL   [3] cap
//   [4, 4 + n OL)                       o_k rows
//   [.., + ceil(n / 32))                reset bitmap, env i = bit i % 32 of word i / 32
//   [.., + ceil(n / 64))                block table: per 64-env pack block, the side slot of its first
//                                       reset (its resets hold consecutive slots, in env order), or
//                                       PACK_DROPPED when the side slab had no room for them
//   [.., + cap (OL + 5))                side entries: local env index, o_0[OL], A[4]
// Side slots are handed out per pack block (never per env): from 16 384 envs on, 3/4 of the capacity
// as 8 regions, one per XCD, each counted by an atomic of its own (hardware XCC_ID), and the rest as
// a shared spill region with one more counter, used when the block's XCD region is full (then the
// other XCDs' regions); below that one shared region.  One counter for all
// blocks serialised at the memory-side atomic unit (~35 ns per atomic on one address: 19.5 us for
// the 512 per-wave atomics of a 32 768-env pack, round 4), eight of them split that queue.
// The counters live in a per-buffer scratch area that is never sent (PACK_SCRATCH_WORDS after the
// largest packed buffer); a pack zeroes the scratch of the buffer the next pack on its stream uses.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cf2 {

constexpr uint32_t XB_PACK = 64;                  // envs per pack block (one block-table word each)
constexpr uint32_t PACK_DROPPED = 0xFFFFFFFFu;     // block-table value: the block's resets got no slot
constexpr uint32_t PACK_XCDS = 8, PACK_CTR_STRIDE = 32;     // counters 128 B apart
constexpr uint32_t PACK_SCRATCH_WORDS = (PACK_XCDS + 1) * PACK_CTR_STRIDE;

struct PackLayout {
    uint32_t n, ol, cap;
    __host__ __device__ uint32_t od() const { return 2u * (ol + 4u); }
    __host__ __device__ uint32_t o_slab() const { return 4u; }
    __host__ __device__ uint32_t bits() const { return 4u + n * ol; }
    __host__ __device__ uint32_t btab() const { return bits() + (n + 31u) / 32u; }
    __host__ __device__ uint32_t side() const { return btab() + (n + XB_PACK - 1u) / XB_PACK; }
    __host__ __device__ uint32_t entry() const { return ol + 5u; }
    __host__ __device__ uint32_t words() const { return (side() + cap * entry() + 3u) & ~3u; }
    // side slots per XCD region (3/4 of the capacity over the 8 regions) and of the spill region.
    // Below 256 pack blocks (16 384 envs) there are few atomics to split, and regions would waste
    // room (a small launch does not spread its blocks over all XCDs): one shared region then.
    __host__ __device__ uint32_t region() const { return n >= 256u * XB_PACK ? (cap * 3u) / (4u * PACK_XCDS) : 0u; }
    __host__ __device__ uint32_t spill() const { return cap - PACK_XCDS * region(); }
};

__device__ __forceinline__ uint32_t pack_xcc_id() {
    return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & (PACK_XCDS - 1u);     // HW_REG XCC_ID
}

// The exchange's pack fused into the env-step (cf2_step_packed): where step_kernel_small writes the
// packed buffer of its envs besides their observation rows
struct PackIO {
    uint32_t* pk;              // packed buffer (null: no pack)
    uint32_t* scratch;         // this buffer's side-slot counters (zeroed by the previous pack)
    uint32_t* next_scratch;    // the counters of the buffer the next pack uses (zeroed here), or null
    uint32_t cap;
};

// The first side slot of a pack block with c > 0 resets (one thread calls it), or PACK_DROPPED:
// the block's XCD region, else the spill region, else the other XCDs' regions (a failed attempt
// leaves that counter past its region, so the region's remaining slots stay unused: the side slab
// overflows only within a few blocks' resets of full).
__device__ __forceinline__ uint32_t pack_alloc(const PackLayout& L, uint32_t* scratch, uint32_t c) {
    const uint32_t x = pack_xcc_id(), r = L.region();
    if (r >= c) {
        const uint32_t old = atomicAdd(scratch + x * PACK_CTR_STRIDE, c);
        if (old + c <= r) return x * r + old;
    }
    const uint32_t old = atomicAdd(scratch + PACK_XCDS * PACK_CTR_STRIDE, c);
    if (old + c <= L.spill()) return PACK_XCDS * r + old;
    if (r >= c) {
        for (uint32_t t = 1; t < PACK_XCDS; ++t) {
            const uint32_t y = (x + t) & (PACK_XCDS - 1u);
            const uint32_t o = atomicAdd(scratch + y * PACK_CTR_STRIDE, c);
            if (o + c <= r) return y * r + o;
        }
    }
    return PACK_DROPPED;
}

// The side slot of local env li (a reset env) from the block table and the bitmap, or PACK_DROPPED.
__device__ __forceinline__ uint32_t pack_slot(const uint32_t* pk, const PackLayout& L, uint32_t li) {
    const uint32_t b = li / XB_PACK, first = pk[L.btab() + b];
    if (first == PACK_DROPPED) return PACK_DROPPED;
    const uint32_t w0 = b * (XB_PACK / 32u), wl = li / 32u;
    uint32_t slot = first;
    for (uint32_t w = w0; w < wl; ++w) slot += (uint32_t)__popc(pk[L.bits() + w]);
    return slot + (uint32_t)__popc(pk[L.bits() + wl] & ((1u << (li % 32u)) - 1u));
}

}  // namespace cf2
