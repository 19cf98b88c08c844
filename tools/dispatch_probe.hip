// Dispatch probe (tools/dispatch_probe.hip): how long a launch of 512 blocks x 256 threads takes to
// start all its waves, per XCD, for a small (16 B) and a large (~1 KB) kernel argument block.
// Each wave stores its XCC id and s_memrealtime (100 MHz) at entry and spins ~20 us so that all
// waves are resident together.  Prints the start spread per XCD and overall.
// build: hipcc --offload-arch=gfx950 -O3 -o build_ab/dispatch_probe tools/dispatch_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>
#include <algorithm>

template <int NB>
struct Big { float f[NB / 4]; };

__device__ __forceinline__ void record(uint64_t* out, float spin) {
    if ((threadIdx.x & 63) == 0) {
        const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);
        const uint64_t t = __builtin_amdgcn_s_memrealtime();
        const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
        out[2 * w] = xcc;
        out[2 * w + 1] = t;
    }
    // keep the wave resident ~20 us
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)spin) __builtin_amdgcn_s_sleep(2);
}
__global__ void __launch_bounds__(256) k_small(uint64_t* out, float spin) { record(out, spin); }
template <int NB>
__global__ void __launch_bounds__(1024) k_big(uint64_t* out, Big<NB> b) { record(out, b.f[3]); }

static void report(const char* name, const std::vector<uint64_t>& h, int waves) {
    uint64_t t0 = UINT64_MAX, t1 = 0;
    uint64_t lo[8], hi[8];
    for (int x = 0; x < 8; ++x) { lo[x] = UINT64_MAX; hi[x] = 0; }
    for (int w = 0; w < waves; ++w) {
        const int x = (int)(h[2 * w] & 7);
        const uint64_t t = h[2 * w + 1];
        t0 = std::min(t0, t); t1 = std::max(t1, t);
        lo[x] = std::min(lo[x], t); hi[x] = std::max(hi[x], t);
    }
    printf("%s: all waves started within %.2f us; per XCD first start (us after the first wave):", name, (t1 - t0) / 100.0);
    for (int x = 0; x < 8; ++x) printf(" %.2f", (lo[x] - t0) / 100.0);
    printf("; per XCD spread:");
    for (int x = 0; x < 8; ++x) printf(" %.2f", (hi[x] - lo[x]) / 100.0);
    printf("\n");
}

template <int NB>
static double spread_us(uint64_t* d, std::vector<uint64_t>& h, int blocks, float spin, int reps, double* tput_us,
                        int threads = 256) {
    Big<NB> b{};
    b.f[3] = spin;
    const int waves = blocks * threads / 64;
    std::vector<double> sp;
    for (int r = 0; r < reps; ++r) {
        hipLaunchKernelGGL(k_big<NB>, dim3(blocks), dim3(threads), 0, 0, d, b);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(h.data(), d, (size_t)waves * 16, hipMemcpyDeviceToHost);
        uint64_t t0 = UINT64_MAX, t1 = 0;
        for (int w = 0; w < waves; ++w) { t0 = std::min(t0, h[2 * w + 1]); t1 = std::max(t1, h[2 * w + 1]); }
        sp.push_back((t1 - t0) / 100.0);
    }
    std::sort(sp.begin(), sp.end());
    // back-to-back launches (no spin): time per launch
    b.f[3] = 0.0f;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(k_big<NB>, dim3(blocks), dim3(threads), 0, 0, d, b);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 200; ++r) hipLaunchKernelGGL(k_big<NB>, dim3(blocks), dim3(threads), 0, 0, d, b);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    *tput_us = ms * 1e3 / 200;
    return sp[sp.size() / 2];
}

int main(int argc, char** argv) {
    const int max_waves = 4096;
    uint64_t* d;
    (void)hipMalloc(&d, (size_t)max_waves * 16);
    std::vector<uint64_t> h((size_t)max_waves * 2);
    if (argc > 1) {
        // sweep: start spread and back-to-back launch time against the number of waves per launch
        // (how much of a short kernel's time the dispatch ramp of its waves is)
        for (int pass = 0; pass < 2; ++pass)
            for (int threads : {256, 64})
                for (int waves : {256, 512, 1024, 2048, 4096}) {
                    double t;
                    const int blocks = waves * 64 / threads;
                    const double sp = spread_us<688>(d, h, blocks, 2000.0f, 11, &t, threads);
                    printf("%4d waves as %4d blocks x %4d threads: median start spread %.2f us, back-to-back %.2f us per launch\n",
                           waves, blocks, threads, sp, t);
                }
        (void)hipFree(d);
        return 0;
    }
    const int waves = 2048;
    for (int pass = 0; pass < 2; ++pass) {
        double t;
        double s16 = spread_us<16>(d, h, 512, 2000.0f, 15, &t);
        printf("kernarg %5d B: median start spread %.2f us, back-to-back %.2f us per launch\n", 16 + 8, s16, t);
        double s688 = spread_us<688>(d, h, 512, 2000.0f, 15, &t);
        printf("kernarg %5d B: median start spread %.2f us, back-to-back %.2f us per launch\n", 688 + 8, s688, t);
        for (int threads : {64, 128, 512, 1024}) {
            const int blocks = waves * 64 / threads;
            double sp = spread_us<688>(d, h, blocks, 2000.0f, 15, &t, threads);
            printf("2048 waves as %4d blocks x %4d threads: median start spread %.2f us, back-to-back %.2f us per launch\n",
                   blocks, threads, sp, t);
        }
    }
    (void)hipFree(d);
    return 0;
}
