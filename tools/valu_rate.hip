// Throughput of a few VALU instructions on gfx950 (tools/valu_rate.hip): every wave runs ITERS
// iterations of 8 independent chains of one instruction; the launch fills every SIMD with 4 waves.
// Prints ns per launch and SIMD cycles per wave-instruction at the measured clock-free rate
// (instructions per SIMD / time, relative to v_fma_f32).
// build: hipcc --offload-arch=gfx950 -O3 -o build_ab/valu_rate tools/valu_rate.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int ITERS = 4096;

__global__ void __launch_bounds__(256) k_fma(float* out, float a, float b) {
    float x[8];
    for (int j = 0; j < 8; ++j) x[j] = threadIdx.x + j;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[j]) : "v"(a), "v"(b));
    float s = 0;
    for (int j = 0; j < 8; ++j) s += x[j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k_mad64(uint64_t* out, uint32_t m) {
    uint64_t x[8];
    for (int j = 0; j < 8; ++j) x[j] = threadIdx.x + j;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            uint32_t lo = (uint32_t)x[j];
            asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, 0" : "=v"(x[j]) : "v"(lo), "v"(m) : "s40", "s41");
        }
    uint64_t s = 0;
    for (int j = 0; j < 8; ++j) s += x[j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k_mullo(uint32_t* out, uint32_t m) {
    uint32_t x[8];
    for (int j = 0; j < 8; ++j) x[j] = threadIdx.x + j;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[j]) : "v"(m));
    uint32_t s = 0;
    for (int j = 0; j < 8; ++j) s += x[j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k_mulhi(uint32_t* out, uint32_t m) {
    uint32_t x[8];
    for (int j = 0; j < 8; ++j) x[j] = threadIdx.x + j;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[j]) : "v"(m));
    uint32_t s = 0;
    for (int j = 0; j < 8; ++j) s += x[j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k_mul24(uint32_t* out, uint32_t m) {
    uint32_t x[8];
    for (int j = 0; j < 8; ++j) x[j] = threadIdx.x + j;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x[j]) : "v"(m));
    uint32_t s = 0;
    for (int j = 0; j < 8; ++j) s += x[j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k_bitop3(uint32_t* out, uint32_t m) {
    uint32_t x[8];
    for (int j = 0; j < 8; ++j) x[j] = threadIdx.x + j;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(x[j]) : "v"(m));
    uint32_t s = 0;
    for (int j = 0; j < 8; ++j) s += x[j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 4;     // 4 blocks of 4 waves per CU: 4 waves per SIMD
    void* buf;
    hipMalloc(&buf, (size_t)blocks * 256 * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double per_simd = (double)ITERS * 8 * 4;   // wave-instructions per SIMD (4 waves)
    auto run = [&](const char* name, auto launch) {
        launch();
        hipDeviceSynchronize();
        hipEventRecord(e0);
        for (int r = 0; r < 10; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double ns = ms * 1e6 / 10;
        printf("%-14s %9.1f us per launch  %6.3f ns per wave-instruction per SIMD\n", name, ns / 1e3, ns / per_simd);
    };
    run("v_fma_f32", [&] { hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(256), 0, 0, (float*)buf, 1.0001f, 0.5f); });
    run("v_bitop3_b32", [&] { hipLaunchKernelGGL(k_bitop3, dim3(blocks), dim3(256), 0, 0, (uint32_t*)buf, 77u); });
    run("v_mul_u32_u24", [&] { hipLaunchKernelGGL(k_mul24, dim3(blocks), dim3(256), 0, 0, (uint32_t*)buf, 77u); });
    run("v_mul_lo_u32", [&] { hipLaunchKernelGGL(k_mullo, dim3(blocks), dim3(256), 0, 0, (uint32_t*)buf, 0xD2511F53u); });
    run("v_mul_hi_u32", [&] { hipLaunchKernelGGL(k_mulhi, dim3(blocks), dim3(256), 0, 0, (uint32_t*)buf, 0xD2511F53u); });
    run("v_mad_u64_u32", [&] { hipLaunchKernelGGL(k_mad64, dim3(blocks), dim3(256), 0, 0, (uint64_t*)buf, 0xD2511F53u); });
    hipFree(buf);
    return 0;
}
