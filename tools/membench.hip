// Memory-side micro-benchmark for the step kernel's access pattern: each env reads R float
// fields and writes W float fields (the persistent state), plus a strided obs-row write.
// Layouts: 0 = SoA (field * N + env), 1 = AoSoA tiles of 64 envs (one contiguous NF*256 B block
// per wave).  Measures what the pattern alone costs on the chip, without the physics.
// build: hipcc --offload-arch=gfx950 -O3 -o membench tools/membench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int LAYOUT, int R, int W, int NF, int OBS>
__global__ void __launch_bounds__(256) kern(const float* __restrict__ in, float* __restrict__ out, float* __restrict__ obs,
                                            uint32_t N, int spin) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    float v[R];
#pragma unroll
    for (int f = 0; f < R; ++f) {
        const size_t idx = LAYOUT == 0 ? (size_t)f * N + i : ((size_t)(i >> 6) * NF + f) * 64 + (i & 63);
        v[f] = in[idx];
    }
    // a dependent arithmetic chain of adjustable length (stand-in for the physics)
    float acc = 0.0f;
#pragma unroll
    for (int f = 0; f < R; ++f) acc += v[f];
    for (int k = 0; k < spin; ++k) acc = acc * 1.0000001f + 1e-7f;
#pragma unroll
    for (int f = 0; f < W; ++f) {
        const size_t idx = LAYOUT == 0 ? (size_t)f * N + i : ((size_t)(i >> 6) * NF + f) * 64 + (i & 63);
        out[idx] = v[f % R] + acc;
    }
    if (OBS) {
        float2* o = reinterpret_cast<float2*>(obs + (size_t)i * OBS);
#pragma unroll
        for (int k = 0; k < OBS / 2; ++k) o[k] = make_float2(v[(2 * k) % R], acc);
    }
}

template <int LAYOUT, int R, int W, int NF, int OBS>
static void run(const char* name, float* in, float* out, float* obs, uint32_t N, int spin) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const dim3 g((N + 255) / 256), blk(256);
    for (int k = 0; k < 10; ++k) hipLaunchKernelGGL((kern<LAYOUT, R, W, NF, OBS>), g, blk, 0, 0, in, out, obs, N, spin);
    CHECK(hipDeviceSynchronize());
    const int iters = 100;
    CHECK(hipEventRecord(a));
    for (int k = 0; k < iters; ++k) hipLaunchKernelGGL((kern<LAYOUT, R, W, NF, OBS>), g, blk, 0, 0, in, out, obs, N, spin);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / iters;
    const double bytes = (double)N * (4.0 * (R + W) + 4.0 * OBS);
    printf("%-34s spin=%4d  %7.1f us  %7.0f GB/s\n", name, spin, us, bytes / (us * 1e-6) / 1e9);
}

int main(int argc, char** argv) {
    const uint32_t N = argc > 1 ? (uint32_t)atoi(argv[1]) : 262144u;
    constexpr int NF = 104;
    float *in, *out, *obs;
    CHECK(hipMalloc(&in, sizeof(float) * NF * N));
    CHECK(hipMalloc(&out, sizeof(float) * NF * N));
    CHECK(hipMalloc(&obs, sizeof(float) * 34 * N));
    CHECK(hipMemset(in, 0, sizeof(float) * NF * N));
    if (argc > 2) {   // calibration mode for the PMC byte counters: one known-byte pattern, few launches
        run<0, 84, 72, NF, 34>("SoA    R84 W72 +obs34 (calib)", in, out, obs, N, 0);
        CHECK(hipFree(in));
        CHECK(hipFree(out));
        CHECK(hipFree(obs));
        return 0;
    }
    const int spins[] = {0, 256, 1024};
    for (int s : spins) {
        run<0, 84, 72, NF, 0>("SoA    R84 W72", in, out, obs, N, s);
        run<1, 84, 72, NF, 0>("AoSoA  R84 W72", in, out, obs, N, s);
        run<0, 84, 72, NF, 34>("SoA    R84 W72 +obs34", in, out, obs, N, s);
        run<1, 84, 72, NF, 34>("AoSoA  R84 W72 +obs34", in, out, obs, N, s);
    }
    run<0, 16, 16, NF, 0>("SoA    R16 W16", in, out, obs, N, 0);
    run<1, 16, 16, NF, 0>("AoSoA  R16 W16", in, out, obs, N, 0);
    CHECK(hipFree(in));
    CHECK(hipFree(out));
    CHECK(hipFree(obs));
    return 0;
}
