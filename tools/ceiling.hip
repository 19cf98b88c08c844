// Memory ceiling of the step kernel's exact access pattern, without the physics: what the
// fastest possible env-step kernel could do on this chip at a given env count.
//   in-place AoSoA state (tiles of 64 envs, NG float4 groups): RG groups read, WG written back
//   + one float4 action row read + a 34-float obs row, a reward and a done byte written.
// Also plain streaming read / write / copy of large buffers for the HBM reference points.
// build: hipcc --offload-arch=gfx950 -O3 -o ceiling tools/ceiling.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int NG = 30;
typedef float f4v __attribute__((ext_vector_type(4)));

template <int RG, int WG>
__global__ void __launch_bounds__(256) step_like(f4v* __restrict__ st, const f4v* __restrict__ act,
                                                 f4v* __restrict__ obs, float* __restrict__ rew,
                                                 unsigned char* __restrict__ done, uint32_t N) {
    __shared__ f4v s_obs[256 * 34 / 4];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    f4v* t = st + (size_t)(i >> 6) * NG * 64 + (i & 63);
    f4v v[RG];
#pragma unroll
    for (int g = 0; g < RG; ++g) v[g] = t[g * 64];
    const f4v a = act[i];
    f4v acc = a;
#pragma unroll
    for (int g = 0; g < RG; ++g) acc += v[g];
#pragma unroll
    for (int g = 0; g < WG; ++g) t[g * 64] = v[g] + acc;
    float* so = reinterpret_cast<float*>(s_obs) + threadIdx.x * 34;
#pragma unroll
    for (int k = 0; k < 34; k += 2) *reinterpret_cast<float2*>(so + k) = make_float2(acc.x + k, acc.y);
    rew[i] = acc.z;
    done[i] = acc.w > 1e30f;
    __syncthreads();
    f4v* dst = obs + (size_t)blockIdx.x * (256 * 34 / 4);
    for (uint32_t k = threadIdx.x; k < 256 * 34 / 4; k += 256) dst[k] = s_obs[k];
}

__global__ void rd(const f4v* __restrict__ a, f4v* __restrict__ out, size_t n) {
    f4v acc = {0, 0, 0, 0};
    for (size_t k = blockIdx.x * 256 + threadIdx.x; k < n; k += (size_t)gridDim.x * 256) acc += a[k];
    if (acc.x == 1234.5f) out[0] = acc;
}
__global__ void wr(f4v* __restrict__ a, size_t n) {
    const f4v z = {1, 2, 3, 4};
    for (size_t k = blockIdx.x * 256 + threadIdx.x; k < n; k += (size_t)gridDim.x * 256) a[k] = z;
}
__global__ void cp(const f4v* __restrict__ a, f4v* __restrict__ b, size_t n) {
    for (size_t k = blockIdx.x * 256 + threadIdx.x; k < n; k += (size_t)gridDim.x * 256) b[k] = a[k];
}
__global__ void rmw(f4v* __restrict__ a, size_t n) {
    for (size_t k = blockIdx.x * 256 + threadIdx.x; k < n; k += (size_t)gridDim.x * 256) a[k] = a[k] * 1.0001f;
}

template <class F>
static double time_us(F launch, int iters) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int k = 0; k < 10; ++k) launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    for (int k = 0; k < iters; ++k) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3 / iters;
}

template <int RG, int WG>
static void run_step(uint32_t N, int act_slabs) {
    f4v *st, *act, *obs;
    float* rew;
    unsigned char* done;
    const size_t tiles = (N + 63) / 64;
    CHECK(hipMalloc(&st, tiles * NG * 1024));
    CHECK(hipMalloc(&act, (size_t)N * 16 * act_slabs));
    CHECK(hipMalloc(&obs, (size_t)N * 136));
    CHECK(hipMalloc(&rew, (size_t)N * 4));
    CHECK(hipMalloc(&done, N));
    CHECK(hipMemset(st, 0, tiles * NG * 1024));
    CHECK(hipMemset(act, 0, (size_t)N * 16 * act_slabs));
    int it = 0;
    const double us = time_us([&] {
        step_like<RG, WG><<<N / 256, 256>>>(st, act + (size_t)(it++ % act_slabs) * N, obs, rew, done, N);
    }, 200);
    const double bytes = (double)N * (16.0 * (RG + WG) + 16 + 136 + 4 + 1);
    printf("step-like N=%8u R%2d W%2d slabs=%d  %7.2f us  %7.0f GB/s (%.1f MB/launch)\n", N, RG, WG, act_slabs, us,
           bytes / (us * 1e-6) / 1e9, bytes / 1e6);
    CHECK(hipFree(st)); CHECK(hipFree(act)); CHECK(hipFree(obs)); CHECK(hipFree(rew)); CHECK(hipFree(done));
}

int main() {
    run_step<22, 17>(262144, 8);
    run_step<22, 17>(262144, 1);
    run_step<20, 15>(262144, 8);
    run_step<18, 13>(262144, 8);
    run_step<22, 17>(65536, 8);
    run_step<22, 17>(1048576, 8);
    run_step<22, 17>(4194304, 8);
    const size_t bytes = (size_t)1 << 30, n = bytes / 16;
    f4v *a, *b;
    CHECK(hipMalloc(&a, bytes));
    CHECK(hipMalloc(&b, bytes));
    CHECK(hipMemset(a, 0, bytes));
    CHECK(hipMemset(b, 0, bytes));
    const int grid = 256 * 32;
    double us = time_us([&] { rd<<<grid, 256>>>(a, b, n); }, 20);
    printf("read  1 GiB            %8.1f us  %7.0f GB/s\n", us, bytes / (us * 1e-6) / 1e9);
    us = time_us([&] { wr<<<grid, 256>>>(a, n); }, 20);
    printf("write 1 GiB            %8.1f us  %7.0f GB/s\n", us, bytes / (us * 1e-6) / 1e9);
    us = time_us([&] { cp<<<grid, 256>>>(a, b, n); }, 20);
    printf("copy  1 GiB            %8.1f us  %7.0f GB/s (r+w)\n", us, 2.0 * bytes / (us * 1e-6) / 1e9);
    us = time_us([&] { rmw<<<grid, 256>>>(a, n); }, 20);
    printf("rmw   1 GiB in place   %8.1f us  %7.0f GB/s (r+w)\n", us, 2.0 * bytes / (us * 1e-6) / 1e9);
    const size_t sm = (size_t)128 << 20, nsm = sm / 16;
    us = time_us([&] { rmw<<<grid, 256>>>(a, nsm); }, 100);
    printf("rmw 128 MiB in place   %8.1f us  %7.0f GB/s (r+w)\n", us, 2.0 * sm / (us * 1e-6) / 1e9);
    CHECK(hipFree(a));
    CHECK(hipFree(b));
    return 0;
}
