// Phase timeline of tblock64_kernel from s_memtime stamps (a TB64_STAMPS build of the
// kernel source; not part of libmvpose).  Build here, run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -o tools/tb64_stamps tools/tb64_stamps.hip
//   ./tools/tb64_stamps [N]
#define TB64_STAMPS 1
#include "../multi-camera_3d_pose_estimation_amd/csrc/tblock64.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

namespace mvp {
void set_error(const char*, ...) {}
[[noreturn]] void fail(int, const char* fmt, ...) {
    va_list a;
    va_start(a, fmt);
    vfprintf(stderr, fmt, a);
    va_end(a);
    fprintf(stderr, "\n");
    exit(1);
}
const uint16_t* conv_zero_region() {
    static uint16_t* z = nullptr;
    if (!z) {
        MVP_HIP(hipMalloc(&z, 65536));
        MVP_HIP(hipMemset(z, 0, 65536));
    }
    return z;
}
}  // namespace mvp

static uint16_t bf16(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16);
}

int main(int argc, char** argv) {
    using G = mvp::B64;
    const int N = argc > 1 ? atoi(argv[1]) : 1024;
    std::mt19937 rng(1);
    std::normal_distribution<float> nd(0.f, 1.f);
    const size_t nx = (size_t)N * 32 * 24 * 64, nw = 64 * 9 * 64;
    std::vector<uint16_t> hx(nx), hw(2 * nw);
    std::vector<float> hb(128);
    for (auto& v : hx) v = bf16(nd(rng));
    for (auto& v : hw) v = bf16(nd(rng) * 0.05f);
    for (auto& v : hb) v = nd(rng) * 0.1f;
    uint16_t *x, *y, *w;
    float* b;
    unsigned long long* st;
    int cus = 0;
    MVP_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int tiles = N * G::TILES_H, grid = std::min(tiles, cus);
    const size_t nst = (size_t)grid * 4 * 4;
    MVP_HIP(hipMalloc(&x, nx * 2));
    MVP_HIP(hipMalloc(&y, nx * 2));
    MVP_HIP(hipMalloc(&w, 2 * nw * 2));
    MVP_HIP(hipMalloc(&b, 128 * 4));
    MVP_HIP(hipMalloc(&st, nst * 8));
    MVP_HIP(hipMemcpy(x, hx.data(), nx * 2, hipMemcpyHostToDevice));
    MVP_HIP(hipMemcpy(w, hw.data(), 2 * nw * 2, hipMemcpyHostToDevice));
    MVP_HIP(hipMemcpy(b, hb.data(), 128 * 4, hipMemcpyHostToDevice));
    MVP_HIP(hipMemset(st, 0, nst * 8));
    MVP_HIP(hipFuncSetAttribute((const void*)mvp::tblock64_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
    mvp::TB64Params p{x, w, b, w + nw, b + 64, y, mvp::conv_zero_region(), N, tiles, st};
    hipEvent_t e0, e1;
    MVP_HIP(hipEventCreate(&e0));
    MVP_HIP(hipEventCreate(&e1));
    for (int i = 0; i < 3; i++) hipLaunchKernelGGL(mvp::tblock64_kernel<false>, dim3(grid), dim3(256), G::LDS, 0, p);
    MVP_HIP(hipEventRecord(e0));
    const int reps = 10;
    for (int i = 0; i < reps; i++) hipLaunchKernelGGL(mvp::tblock64_kernel<false>, dim3(grid), dim3(256), G::LDS, 0, p);
    MVP_HIP(hipEventRecord(e1));
    MVP_HIP(hipEventSynchronize(e1));
    float ms = 0;
    MVP_HIP(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> h(nst);
    MVP_HIP(hipMemcpy(h.data(), st, nst * 8, hipMemcpyDeviceToHost));
    printf("N=%d grid=%d tiles=%d: %.1f us per launch (stamped build)\n", N, grid, tiles, ms * 1000 / reps);
    // per wave: s_memtime segment sums over the launch's phases (the last launch), per phase
    const int phases = tiles / grid;  // tiles per workgroup (crop ranges: 4 per crop)
    auto med = [](std::vector<double> v) {
        std::sort(v.begin(), v.end());
        return v.empty() ? 0.0 : v[v.size() / 2];
    };
    const char* c1[3] = {"k-loop (+ half A epilogues)", "half B epilogue", "barrier wait (+ next row copy)"};
    const char* c2[4] = {"setup + k-loop (+ DMA, half A epilogues)", "half B epilogue", "halo vmcnt wait",
                         "barrier wait"};
    for (int role = 0; role < 2; role++) {
        printf("%s waves, cycles per phase (median over workgroups):\n", role ? "conv2" : "conv1");
        double tot = 0;
        for (int i = 0; i < (role ? 4 : 3); i++) {
            std::vector<double> v;
            for (int blk = 0; blk < grid; blk++)
                for (int w = 2 * role; w < 2 * role + 2; w++) v.push_back((double)h[(blk * 4 + w) * 4 + i] / phases);
            const double m = med(v);
            tot += m;
            printf("  %-44s %8.0f\n", role ? c2[i] : c1[i], m);
        }
        printf("  %-44s %8.0f\n", "sum", tot);
    }
    printf("ideal MFMA cycles per wave per phase: 216 x 32 = 6912 (tiles 1-3), conv1 288 x 32 = 9216 (first tile)\n");
    return 0;
}
