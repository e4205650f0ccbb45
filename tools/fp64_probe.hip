// Issue-rate probe for the VALU instruction mix of the triangulation kernels: wave64
// v_fma_f64 / v_mul_f64 / v_add_f64 / v_fma_f32 / v_rcp_f64 streams, 8 independent chains
// per lane, every CU busy (2,048 workgroups of 256 threads, 8 waves per SIMD).  Prints the
// issue cycles per wave-instruction per SIMD at the measured clock-free rate
// (cycles = time x 2.4 GHz x 1,024 SIMDs / wave-instructions).
//   hipcc --offload-arch=gfx950 -O3 tools/fp64_probe.hip -o tools/fp64_probe && ./tools/fp64_probe
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 4096, kChains = 8, kBlocks = 2048, kThreads = 256;

template <int OP>
__global__ __launch_bounds__(256) void probe(double* out, double a, double b) {
    double x[kChains];
    float xf[kChains];
#pragma unroll
    for (int c = 0; c < kChains; c++) {
        x[c] = threadIdx.x * 1e-3 + c;
        xf[c] = (float)x[c];
    }
    for (int i = 0; i < kIters; i++) {
#pragma unroll
        for (int c = 0; c < kChains; c++) {
            if constexpr (OP == 0) x[c] = __builtin_fma(x[c], a, b);
            if constexpr (OP == 1) x[c] = x[c] * a;
            if constexpr (OP == 2) x[c] = x[c] + b;
            if constexpr (OP == 3) xf[c] = __builtin_fmaf(xf[c], (float)a, (float)b);
            if constexpr (OP == 4) x[c] = __builtin_amdgcn_rcp(x[c]);
        }
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < kChains; c++) s += x[c] + xf[c];
    if (s == 12345.678) out[0] = s;  // keep the chains alive
}

template <int OP>
double run(const char* name, double* d) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(probe<OP>, dim3(kBlocks), dim3(kThreads), 0, 0, d, 0.999999, 1e-9);
    hipEventRecord(e0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(probe<OP>, dim3(kBlocks), dim3(kThreads), 0, 0, d, 0.999999, 1e-9);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    const double winst = (double)kBlocks * (kThreads / 64) * kIters * kChains;
    const double cyc = ms * 1e-3 * 2.4e9 * 1024 / winst;
    printf("%-10s %8.3f ms  %6.2f cycles per wave64 instruction per SIMD (at 2.4 GHz)\n", name, ms, cyc);
    return cyc;
}

int main() {
    double* d;
    hipMalloc(&d, 8);
    run<0>("v_fma_f64", d);
    run<1>("v_mul_f64", d);
    run<2>("v_add_f64", d);
    run<3>("v_fma_f32", d);
    run<4>("v_rcp_f64", d);
    hipFree(d);
    return 0;
}
