// HBM rate probe (tools/hbm_probe.hip): read-only, write-only and copy kernels over 2 GiB buffers
// (far beyond the 256 MB Infinity Cache), plain and non-temporal, at several grid sizes.
// build: hipcc --offload-arch=gfx950 -O3 -o build_ab/hbm_probe tools/hbm_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

template <bool NT, int UNROLL>
__global__ void __launch_bounds__(256) k_copy(const u4* __restrict__ s, u4* __restrict__ d, size_t n) {
    const size_t stride = (size_t)gridDim.x * 256u;
    size_t i = (size_t)blockIdx.x * 256u + threadIdx.x;
    for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
        u4 v[UNROLL];
#pragma unroll
        for (int k = 0; k < UNROLL; ++k) v[k] = NT ? __builtin_nontemporal_load(s + i + k * stride) : s[i + k * stride];
#pragma unroll
        for (int k = 0; k < UNROLL; ++k) {
            if (NT) __builtin_nontemporal_store(v[k], d + i + k * stride);
            else d[i + k * stride] = v[k];
        }
    }
    for (; i < n; i += stride) d[i] = s[i];
}
template <bool NT, int UNROLL>
__global__ void __launch_bounds__(256) k_read(const u4* __restrict__ s, u4* __restrict__ out, size_t n) {
    const size_t stride = (size_t)gridDim.x * 256u;
    size_t i = (size_t)blockIdx.x * 256u + threadIdx.x;
    u4 acc = {0, 0, 0, 0};
    for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
#pragma unroll
        for (int k = 0; k < UNROLL; ++k) acc ^= NT ? __builtin_nontemporal_load(s + i + k * stride) : s[i + k * stride];
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[threadIdx.x] = acc;
}
template <bool NT>
__global__ void __launch_bounds__(256) k_write(u4* __restrict__ d, size_t n) {
    const size_t stride = (size_t)gridDim.x * 256u;
    const u4 v = {1u, 2u, 3u, (unsigned)threadIdx.x};
    for (size_t i = (size_t)blockIdx.x * 256u + threadIdx.x; i < n; i += stride) {
        if (NT) __builtin_nontemporal_store(v, d + i);
        else d[i] = v;
    }
}

int main() {
    const size_t bytes = (size_t)2 << 30, n = bytes / 16;
    u4 *a, *b;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
    (void)hipMemset(a, 1, bytes);
    (void)hipMemset(b, 0, bytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    auto timeit = [&](const char* name, double traffic, auto launch) {
        for (int r = 0; r < 3; ++r) launch();
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0);
        for (int r = 0; r < 10; ++r) launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-34s %8.1f GB/s\n", name, traffic * 10 / (ms * 1e-3) / 1e9);
    };
    for (int per : {4, 8, 16}) {
        const dim3 g(cus * per);
        char nm[64];
        snprintf(nm, sizeof nm, "copy nt u4 x4, %d blk/CU", per);
        timeit(nm, 2.0 * bytes, [&] { hipLaunchKernelGGL((k_copy<true, 4>), g, dim3(256), 0, 0, a, b, n); });
        snprintf(nm, sizeof nm, "copy plain u4 x4, %d blk/CU", per);
        timeit(nm, 2.0 * bytes, [&] { hipLaunchKernelGGL((k_copy<false, 4>), g, dim3(256), 0, 0, a, b, n); });
        snprintf(nm, sizeof nm, "copy plain u4 x8, %d blk/CU", per);
        timeit(nm, 2.0 * bytes, [&] { hipLaunchKernelGGL((k_copy<false, 8>), g, dim3(256), 0, 0, a, b, n); });
        snprintf(nm, sizeof nm, "read plain u4 x8, %d blk/CU", per);
        timeit(nm, 1.0 * bytes, [&] { hipLaunchKernelGGL((k_read<false, 8>), g, dim3(256), 0, 0, a, b, n); });
        snprintf(nm, sizeof nm, "read nt u4 x8, %d blk/CU", per);
        timeit(nm, 1.0 * bytes, [&] { hipLaunchKernelGGL((k_read<true, 8>), g, dim3(256), 0, 0, a, b, n); });
        snprintf(nm, sizeof nm, "write plain u4, %d blk/CU", per);
        timeit(nm, 1.0 * bytes, [&] { hipLaunchKernelGGL((k_write<false>), g, dim3(256), 0, 0, b, n); });
        snprintf(nm, sizeof nm, "write nt u4, %d blk/CU", per);
        timeit(nm, 1.0 * bytes, [&] { hipLaunchKernelGGL((k_write<true>), g, dim3(256), 0, 0, b, n); });
    }
    (void)hipFree(a);
    (void)hipFree(b);
    return 0;
}
