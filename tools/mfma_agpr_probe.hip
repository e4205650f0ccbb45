// MFMA issue rate with the A operand in AGPRs vs VGPRs (v_mfma_f32_32x32x16_bf16, one wave
// per SIMD, 4 independent accumulators in AGPRs), the question tblock64's two-cout-group form
// raised (its weights are split over both files).  Build here, run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/mfma_agpr_probe tools/mfma_agpr_probe.hip
//   ./tools/mfma_agpr_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

template <bool A_IN_AGPR>
__global__ __launch_bounds__(256, 1) void probe(const bf16x8* in, float* out, int iters, long long* cyc) {
    const int lane = threadIdx.x & 63;
    bf16x8 a0 = in[lane], a1 = in[64 + lane], b0 = in[128 + lane], b1 = in[192 + lane];
    f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
        if constexpr (A_IN_AGPR) {
            asm volatile(
                "v_mfma_f32_32x32x16_bf16 %0, %4, %6, %0\n\t"
                "v_mfma_f32_32x32x16_bf16 %1, %5, %6, %1\n\t"
                "v_mfma_f32_32x32x16_bf16 %2, %4, %7, %2\n\t"
                "v_mfma_f32_32x32x16_bf16 %3, %5, %7, %3"
                : "+a"(c0), "+a"(c1), "+a"(c2), "+a"(c3)
                : "a"(a0), "a"(a1), "v"(b0), "v"(b1));
        } else {
            asm volatile(
                "v_mfma_f32_32x32x16_bf16 %0, %4, %6, %0\n\t"
                "v_mfma_f32_32x32x16_bf16 %1, %5, %6, %1\n\t"
                "v_mfma_f32_32x32x16_bf16 %2, %4, %7, %2\n\t"
                "v_mfma_f32_32x32x16_bf16 %3, %5, %7, %3"
                : "+a"(c0), "+a"(c1), "+a"(c2), "+a"(c3)
                : "v"(a0), "v"(a1), "v"(b0), "v"(b1));
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 16; e++) s += c0[e] + c1[e] + c2[e] + c3[e];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    bf16x8* in;
    float* out;
    long long* cyc;
    CHECK(hipMalloc(&in, 256 * sizeof(bf16x8)));
    CHECK(hipMemset(in, 0, 256 * sizeof(bf16x8)));
    CHECK(hipMalloc(&out, (size_t)cus * 256 * 4));
    CHECK(hipMalloc(&cyc, cus * 8));
    const int iters = 20000;
    for (int rep = 0; rep < 2; rep++)
        for (int v = 0; v < 2; v++) {
            hipEvent_t e0, e1;
            CHECK(hipEventCreate(&e0));
            CHECK(hipEventCreate(&e1));
            CHECK(hipEventRecord(e0));
            if (v)
                hipLaunchKernelGGL(probe<true>, dim3(cus), dim3(256), 0, 0, in, out, iters, cyc);
            else
                hipLaunchKernelGGL(probe<false>, dim3(cus), dim3(256), 0, 0, in, out, iters, cyc);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            long long c = 0;
            CHECK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
            printf("A in %s: %.3f ms, %.2f cycles per MFMA (block 0), %.1f TFLOP/s\n", v ? "AGPR" : "VGPR", ms,
                   (double)c / (4.0 * iters), 2.0 * 32 * 32 * 16 * 4.0 * iters * 4 * cus / (ms * 1e-3) / 1e12);
        }
    return 0;
}
