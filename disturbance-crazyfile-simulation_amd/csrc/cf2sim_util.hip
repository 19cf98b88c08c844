// cf2sim_util.hip -- measurement support for bench.py (not on the env-step path).
//
// cf2_hbm_probe: streaming kernels bench.py times on 2 GiB buffers to measure the box's own HBM
// rates (the peak re-measured with a STREAM-style kernel), the denominators of
// roofline.out_of_cache.frac_of_measured_hbm.  16 B per lane per access, grid-strided over 16
// blocks per CU, non-temporal loads and stores (tools/hbm_probe.hip measured the variants: nt
// reads at 16 blocks per CU are the fastest read stream, ~6.0 TB/s; copies reach ~4.8 TB/s).
//   mode 0: copy src -> dst (bytes read + bytes written)
//   mode 1: read src (8 accesses in flight per lane), XOR-reduced; dst receives nothing unless the
//           reduction hits a sentinel (it keeps the loads alive)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/cf2sim.h"
#include "cf2sim_internal.h"

namespace cf2 {

typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) hbm_copy_kernel(const u32x4v* __restrict__ src, u32x4v* __restrict__ dst,
                                                       size_t n16) {
    const size_t stride = (size_t)gridDim.x * 256u;
    size_t i = (size_t)blockIdx.x * 256u + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        u32x4v v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = __builtin_nontemporal_load(src + i + k * stride);
#pragma unroll
        for (int k = 0; k < 4; ++k) __builtin_nontemporal_store(v[k], dst + i + k * stride);
    }
    for (; i < n16; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

__global__ void __launch_bounds__(256) hbm_read_kernel(const u32x4v* __restrict__ src, u32x4v* __restrict__ dst,
                                                       size_t n16) {
    const size_t stride = (size_t)gridDim.x * 256u;
    size_t i = (size_t)blockIdx.x * 256u + threadIdx.x;
    u32x4v acc = {0u, 0u, 0u, 0u};
    for (; i + 7 * stride < n16; i += 8 * stride) {
#pragma unroll
        for (int k = 0; k < 8; ++k) acc ^= __builtin_nontemporal_load(src + i + k * stride);
    }
    for (; i < n16; i += stride) acc ^= __builtin_nontemporal_load(src + i);
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) dst[threadIdx.x] = acc;
}

}  // namespace cf2

extern "C" int cf2_hbm_probe(void* dst_dev, const void* src_dev, size_t bytes, int mode, void* stream) {
    if (!dst_dev || !src_dev || (bytes & 15u) || ((uintptr_t)dst_dev & 15u) || ((uintptr_t)src_dev & 15u) ||
        (mode != 0 && mode != 1) || (mode == 1 && bytes < 256u * 16u))
        return CF2_ERR_INVALID_ARG;
    if (bytes == 0) return CF2_OK;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const dim3 grid((unsigned)cus * 16u), block(256);
    const auto* s = static_cast<const cf2::u32x4v*>(src_dev);
    auto* d = static_cast<cf2::u32x4v*>(dst_dev);
    if (mode == 0) hipLaunchKernelGGL(cf2::hbm_copy_kernel, grid, block, 0, (hipStream_t)stream, s, d, bytes / 16u);
    else hipLaunchKernelGGL(cf2::hbm_read_kernel, grid, block, 0, (hipStream_t)stream, s, d, bytes / 16u);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? CF2_OK : cf2::hip_fail(e);
}
