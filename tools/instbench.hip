// Issue cost of the instructions the RNG is built from, one wave per SIMD and 2 waves per SIMD:
// 8 independent chains per lane, cycles per instruction from s_memtime.
// build: hipcc --offload-arch=gfx950 -O3 -o build_ab/instbench tools/instbench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s\n", hipGetErrorString(e_)); return 1; } } while (0)

enum { ITERS = 256, CH = 8 };

template <int OP>
__global__ void kern(uint32_t* out, uint64_t* cycles, uint32_t seed) {
    uint32_t a[CH], b[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) { a[c] = seed * (threadIdx.x + 7 * c + 1); b[c] = a[c] ^ 0x9E3779B9u; }
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < ITERS; ++k) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            if (OP == 0) {          // v_mad_u64_u32 (32x32 -> 64)
                const uint64_t p = (uint64_t)0xD2511F53u * a[c];
                a[c] = (uint32_t)(p >> 32) ^ (uint32_t)p;
            } else if (OP == 1) {   // v_mul_hi_u32 + v_mul_lo_u32
                const uint32_t hi = __umulhi(0xD2511F53u, a[c]), lo = 0xD2511F53u * a[c];
                a[c] = hi ^ lo;
            } else if (OP == 2) {   // v_xor_b32 x2
                a[c] = (a[c] ^ b[c]) ^ 0x1234567u;
            } else if (OP == 3) {   // v_fma_f32
                float f = __uint_as_float(a[c] & 0x3fffffffu);
                f = __builtin_fmaf(f, 1.0001f, 0.5f);
                a[c] = __float_as_uint(f);
            } else {                // v_log_f32 + v_sqrt_f32 (transcendental pair)
                float f = __uint_as_float((a[c] & 0x007fffffu) | 0x3f800000u);
                f = __builtin_amdgcn_sqrtf(__builtin_amdgcn_logf(f) + 2.0f);
                a[c] = __float_as_uint(f);
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) r ^= a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if (threadIdx.x == 0) cycles[blockIdx.x] = t1 - t0;
}

template <int OP>
static int run(const char* name, int insts_per_op, int waves_per_simd) {
    uint32_t* out; uint64_t* cyc;
    const int blocks = 256 * waves_per_simd;   // 256 CUs; a 256-thread block = one wave per SIMD
    CHECK(hipMalloc(&out, sizeof(uint32_t) * blocks * 256));
    CHECK(hipMalloc(&cyc, sizeof(uint64_t) * blocks));
    hipLaunchKernelGGL((kern<OP>), dim3(blocks), dim3(256), 0, 0, out, cyc, 12345u);
    CHECK(hipDeviceSynchronize());
    uint64_t h[4096];
    CHECK(hipMemcpy(h, cyc, sizeof(uint64_t) * blocks, hipMemcpyDeviceToHost));
    double s = 0; for (int k = 0; k < blocks; ++k) s += (double)h[k];
    s /= blocks;
    // s_memtime counts at the shader clock (MI355X_MICROARCH.md constants table)
    printf("%-28s waves/SIMD=%d  %6.2f cycles per instruction per wave\n", name, waves_per_simd,
           s / ((double)ITERS * CH * insts_per_op));
    CHECK(hipFree(out)); CHECK(hipFree(cyc));
    return 0;
}

int main() {
    for (int w = 1; w <= 2; ++w) {
        run<0>("v_mad_u64_u32 (+xor)", 2, w);
        run<1>("v_mul_hi/lo_u32 (+xor)", 3, w);
        run<2>("v_xor_b32", 2, w);
        run<3>("v_fma_f32 (+and)", 2, w);
        run<4>("v_log+v_sqrt (+add,or,and)", 5, w);
    }
    return 0;
}
