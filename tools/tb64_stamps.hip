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
    const size_t nst = (size_t)grid * 4 * 16 * 4;
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
    // per role, per segment: median over blocks, phases 2..13
    auto at = [&](int blk, int wave, int k, int i) { return (long long)h[((blk * 4 + wave) * 16 + k) * 4 + i]; };
    // per tile kind: s = k % 4 == 0 (conv1 computes all 10 rows: 8 fragments) and s > 0 (rows 2-9: 6)
    auto med = [](std::vector<long long> v) {
        std::sort(v.begin(), v.end());
        return v.empty() ? 0LL : v[v.size() / 2];
    };
    for (int kind = 0; kind < 2; kind++) {
        std::vector<long long> c1_mfma, c1_epi, c1_bar, c2_mfma, c2_epi, c2_dma, c2_bar, phase;
        for (int blk = 0; blk < grid; blk++)
            for (int k = 2; k < 14; k++) {
                if ((k % G::TILES_H == 0) != (kind == 0)) continue;
                for (int wv = 0; wv < 2; wv++) {
                    c1_mfma.push_back(at(blk, wv, k, 1) - at(blk, wv, k, 0));
                    c1_epi.push_back(at(blk, wv, k, 2) - at(blk, wv, k, 1));
                    c1_bar.push_back(at(blk, wv, k + 1, 0) - at(blk, wv, k, 2));
                }
                phase.push_back(at(blk, 0, k + 1, 0) - at(blk, 0, k, 0));
                for (int wv = 2; wv < 4; wv++) {
                    c2_mfma.push_back(at(blk, wv, k, 1) - at(blk, wv, k, 0));
                    c2_epi.push_back(at(blk, wv, k, 2) - at(blk, wv, k, 1));
                    c2_dma.push_back(at(blk, wv, k, 3) - at(blk, wv, k, 2));
                    c2_bar.push_back(at(blk, wv, k + 1, 0) - at(blk, wv, k, 3));
                }
            }
        printf("%s: phase %lld cycles (s_memtime ticks)\n", kind == 0 ? "first tile of a crop (8 conv1 fragments)"
                                                                        : "tiles 1-3 (6 conv1 fragments)",
               med(phase));
        printf("  conv1: mfma loop %lld, epilogue %lld, barrier wait %lld\n", med(c1_mfma), med(c1_epi), med(c1_bar));
        printf("  conv2: setup+mfma %lld, residual wait+epilogue %lld, dma wait %lld, barrier wait %lld\n",
               med(c2_mfma), med(c2_epi), med(c2_dma), med(c2_bar));
    }
    // the tick rate: the whole launch over the per-block sum of phases
    {
        std::vector<long long> span;
        for (int blk = 0; blk < grid; blk++) span.push_back(at(blk, 0, 15, 0) - at(blk, 0, 1, 0));
        std::sort(span.begin(), span.end());
        printf("phases 1-15 of block median: %lld ticks\n", span[span.size() / 2]);
    }
    printf("ideal per phase: 216 MFMAs x 32 = %d cycles (tiles 1-3), conv1 288 x 32 = %d (first tile)\n", 216 * 32, 288 * 32);
    return 0;
}
