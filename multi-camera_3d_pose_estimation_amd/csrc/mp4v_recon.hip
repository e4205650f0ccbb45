// Device half of the split MPEG-4 Part 2 decode (mp4v.h): reconstructs VOPs from the host's
// macroblock records and inverse-quantised coefficients — FFmpeg's simple IDCT (the host
// decoder's idct_row / idct_col, integer-exact), half-pel motion compensation with
// vop_rounding_type and edge clamping, I420 -> BGR24 (BT.601 limited range, the host
// bgr_rows arithmetic) — bit-identical to mp4v.cpp's own reconstruction, which
// tests/test_mp4v_gpu.py asserts frame by frame.
//
// Replaces the pixel half of cv.VideoCapture's decode of the reference's mp4v recordings
// (utils.py:849-909, written by synchronize_videos.py:64,240); the decoded frames land in
// HBM, where the 2D stage reads them, instead of crossing PCIe as 2.76 MB BGR frames.
//
// One workgroup (64 threads) per (macroblock, job): a job is one VOP of one stream slot (a GOP
// decodes in its own slot; GOPs are independent, so a launch reconstructs one VOP of every
// slot).  Luma and chroma land in the slot's `cur` picture; the macroblock's 16 x 16 BGR pixels
// (cropped to the frame) go to the job's output frame.  Bytes per macroblock: 384 picture
// bytes written, <= 384 prediction bytes read (+ clamped edges), 768 BGR bytes written, the
// record (32 B) and the coefficient entries (4 B each): HBM-bound work of ~1.6 KB per
// macroblock, 5.6 MB per 1280x720 frame.
#include <hip/hip_runtime.h>

#include "mp4v.h"
#include "mvp_common.h"

namespace {

using mp4v::Job;
using mp4v::MbRec;

constexpr int W1 = 22725, W2 = 21407, W3 = 19266, W4 = 16383, W5 = 12873, W6 = 8867, W7 = 4520;
constexpr int ROW_SHIFT = 11, COL_SHIFT = 20;

__device__ __forceinline__ void idct_row(int16_t* r) {
    if (!(r[1] | r[2] | r[3] | r[4] | r[5] | r[6] | r[7])) {
        const int16_t v = (int16_t)(uint16_t)((r[0] * 8) & 0xffff);
        for (int i = 0; i < 8; i++) r[i] = v;
        return;
    }
    int a0 = W4 * r[0] + (1 << (ROW_SHIFT - 1));
    int a1 = a0, a2 = a0, a3 = a0;
    a0 += W2 * r[2];
    a1 += W6 * r[2];
    a2 -= W6 * r[2];
    a3 -= W2 * r[2];
    int b0 = W1 * r[1] + W3 * r[3];
    int b1 = W3 * r[1] - W7 * r[3];
    int b2 = W5 * r[1] - W1 * r[3];
    int b3 = W7 * r[1] - W5 * r[3];
    if (r[4] | r[5] | r[6] | r[7]) {
        a0 += W4 * r[4] + W6 * r[6];
        a1 += -W4 * r[4] - W2 * r[6];
        a2 += -W4 * r[4] + W2 * r[6];
        a3 += W4 * r[4] - W6 * r[6];
        b0 += W5 * r[5] + W7 * r[7];
        b1 += -W1 * r[5] - W5 * r[7];
        b2 += W7 * r[5] + W3 * r[7];
        b3 += W3 * r[5] - W1 * r[7];
    }
    r[0] = (int16_t)((a0 + b0) >> ROW_SHIFT);
    r[7] = (int16_t)((a0 - b0) >> ROW_SHIFT);
    r[1] = (int16_t)((a1 + b1) >> ROW_SHIFT);
    r[6] = (int16_t)((a1 - b1) >> ROW_SHIFT);
    r[2] = (int16_t)((a2 + b2) >> ROW_SHIFT);
    r[5] = (int16_t)((a2 - b2) >> ROW_SHIFT);
    r[3] = (int16_t)((a3 + b3) >> ROW_SHIFT);
    r[4] = (int16_t)((a3 - b3) >> ROW_SHIFT);
}

// the host's idct_col; its DC-only-rows shortcut computes the same values (every column then
// reduces to the c[0] term), so the device always takes the full column pass
__device__ __forceinline__ void idct_col(const int16_t* c, int (&o)[8]) {
    int a0 = W4 * (c[0] + ((1 << (COL_SHIFT - 1)) / W4));
    int a1 = a0, a2 = a0, a3 = a0;
    a0 += W2 * c[16];
    a1 += W6 * c[16];
    a2 -= W6 * c[16];
    a3 -= W2 * c[16];
    int b0 = W1 * c[8] + W3 * c[24];
    int b1 = W3 * c[8] - W7 * c[24];
    int b2 = W5 * c[8] - W1 * c[24];
    int b3 = W7 * c[8] - W5 * c[24];
    a0 += W4 * c[32];
    a1 -= W4 * c[32];
    a2 -= W4 * c[32];
    a3 += W4 * c[32];
    b0 += W5 * c[40];
    b1 -= W1 * c[40];
    b2 += W7 * c[40];
    b3 += W3 * c[40];
    a0 += W6 * c[48];
    a1 -= W2 * c[48];
    a2 += W2 * c[48];
    a3 -= W6 * c[48];
    b0 += W7 * c[56];
    b1 -= W5 * c[56];
    b2 += W3 * c[56];
    b3 -= W1 * c[56];
    o[0] = (a0 + b0) >> COL_SHIFT;
    o[1] = (a1 + b1) >> COL_SHIFT;
    o[2] = (a2 + b2) >> COL_SHIFT;
    o[3] = (a3 + b3) >> COL_SHIFT;
    o[4] = (a3 - b3) >> COL_SHIFT;
    o[5] = (a2 - b2) >> COL_SHIFT;
    o[6] = (a1 - b1) >> COL_SHIFT;
    o[7] = (a0 - b0) >> COL_SHIFT;
}

__device__ __forceinline__ int clip8(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }

struct ReconParams {
    const Job* jobs;
    int width, height, mb_w, mb_h;
};

// Half-pel prediction of one pixel: the host mc() reads a (w + 1) x (h + 1) window straight from
// the plane when it lies inside the visible vw x vh picture and with clamped coordinates
// otherwise; clamping is the identity inside, so per-pixel clamping gives the same bytes.
__device__ __forceinline__ int mc_pixel(const uint8_t* ref, int pw, int vw, int vh, int x, int y, int mvx, int mvy,
                                        int rnd) {
    const int sx = x + (mvx >> 1), sy = y + (mvy >> 1);
    const int hx = mvx & 1, hy = mvy & 1;
    const int x0 = min(max(sx, 0), vw - 1), x1 = min(max(sx + 1, 0), vw - 1);
    const int y0 = min(max(sy, 0), vh - 1), y1 = min(max(sy + 1, 0), vh - 1);
    const int a = ref[y0 * pw + x0];
    if (!hx && !hy) return a;
    if (hx && !hy) return (a + ref[y0 * pw + x1] + 1 - rnd) >> 1;
    if (!hx && hy) return (a + ref[y1 * pw + x0] + 1 - rnd) >> 1;
    return (a + ref[y0 * pw + x1] + ref[y1 * pw + x0] + ref[y1 * pw + x1] + 2 - rnd) >> 2;
}

__global__ __launch_bounds__(64) void mp4v_recon_kernel(ReconParams p) {
    const Job job = p.jobs[blockIdx.y];
    const int mb = blockIdx.x;
    const int mb_x = mb % p.mb_w, mb_y = mb / p.mb_w;
    const int t = threadIdx.x;
    const int pw = p.mb_w * 16, ph = p.mb_h * 16, cw = p.mb_w * 8, ch = p.mb_h * 8;
    uint8_t* cur = job.cur;
    __shared__ int16_t blk[6][64];
    __shared__ uint8_t pix_y[16][16], pix_u[8][8], pix_v[8][8];
    const MbRec* rp = job.rec + mb;
    const int kind = job.coded ? rp->kind : mp4v::MB_LOST;
    if (kind == mp4v::MB_LOST) {
        // not-coded VOP or a macroblock no video packet reached: the picture as it stands
        for (int i = t; i < 384; i += 64) {
            if (i < 256) pix_y[i >> 4][i & 15] = cur[(size_t)(16 * mb_y + (i >> 4)) * pw + 16 * mb_x + (i & 15)];
            else {
                const int j = i - 256, c = j >> 6, q = j & 63;
                const uint8_t* pl = cur + (size_t)pw * ph + (size_t)c * cw * ch;
                (c ? pix_v : pix_u)[q >> 3][q & 7] = pl[(size_t)(8 * mb_y + (q >> 3)) * cw + 8 * mb_x + (q & 7)];
            }
        }
    } else {
        // coefficients -> LDS blocks
        for (int i = t; i < 6 * 64; i += 64) (&blk[0][0])[i] = 0;
        __syncthreads();
        if (kind != mp4v::MB_COPY) {
            int off = 0;
            for (int n = 0; n < 6; n++) {
                const int cnt = rp->nnz[n];
                for (int i = t; i < cnt; i += 64) {
                    const uint32_t e = job.coef[rp->coef + off + i];
                    blk[n][e >> 16] = (int16_t)(uint16_t)(e & 0xffff);
                }
                off += cnt;
            }
        }
        __syncthreads();
        if (t < 48) idct_row(&blk[t >> 3][8 * (t & 7)]);
        __syncthreads();
        if (t < 48) {
            const int n = t >> 3, c = t & 7;
            int o[8];
            idct_col(&blk[n][c], o);
            const bool luma = n < 4;
            const int bx = luma ? 16 * mb_x + 8 * (n & 1) + c : 8 * mb_x + c;
            const int by0 = luma ? 16 * mb_y + 8 * (n >> 1) : 8 * mb_y;
            const uint8_t* ref = luma ? job.ref : job.ref + (size_t)pw * ph + (size_t)(n - 4) * cw * ch;
            const int rw = luma ? pw : cw;
            const int vw = luma ? p.width : (p.width + 1) >> 1, vh = luma ? p.height : (p.height + 1) >> 1;
            const int mvx = kind == mp4v::MB_INTER ? (luma ? rp->mv[n][0] : rp->cmv[0]) : 0;
            const int mvy = kind == mp4v::MB_INTER ? (luma ? rp->mv[n][1] : rp->cmv[1]) : 0;
            for (int r = 0; r < 8; r++) {
                int v;
                if (kind == mp4v::MB_INTRA) v = clip8(o[r]);
                else v = clip8(mc_pixel(ref, rw, vw, vh, bx, by0 + r, mvx, mvy, job.rounding) + o[r]);
                if (luma) pix_y[8 * (n >> 1) + r][8 * (n & 1) + c] = (uint8_t)v;
                else (n == 4 ? pix_u : pix_v)[r][c] = (uint8_t)v;
            }
        }
        __syncthreads();
        // the picture (every byte of the macroblock, MB-aligned planes)
        for (int i = t; i < 384; i += 64) {
            if (i < 256) cur[(size_t)(16 * mb_y + (i >> 4)) * pw + 16 * mb_x + (i & 15)] = pix_y[i >> 4][i & 15];
            else {
                const int j = i - 256, c = j >> 6, q = j & 63;
                uint8_t* pl = cur + (size_t)pw * ph + (size_t)c * cw * ch;
                pl[(size_t)(8 * mb_y + (q >> 3)) * cw + 8 * mb_x + (q & 7)] = (c ? pix_v : pix_u)[q >> 3][q & 7];
            }
        }
    }
    __syncthreads();
    if (!job.bgr) return;
    // BGR24, BT.601 limited range (mp4v.cpp bgr_rows): c = 298 Y, then the 2 x 2 quad's chroma terms
    for (int i = t; i < 256; i += 64) {
        const int yy = i >> 4, xx = i & 15;
        const int y = 16 * mb_y + yy, x = 16 * mb_x + xx;
        if (y >= p.height || x >= p.width) continue;
        const int u = pix_u[yy >> 1][xx >> 1] - 128, v = pix_v[yy >> 1][xx >> 1] - 128;
        const int c = 298 * pix_y[yy][xx];
        uint8_t* o = job.bgr + ((size_t)y * p.width + x) * 3;
        o[0] = (uint8_t)clip8((c + 516 * u + 128 - 298 * 16) >> 8);
        o[1] = (uint8_t)clip8((c - 100 * u - 208 * v + 128 - 298 * 16) >> 8);
        o[2] = (uint8_t)clip8((c + 409 * v + 128 - 298 * 16) >> 8);
    }
}

}  // namespace

extern "C" int mvp_mp4v_reconstruct(const void* jobs_dev, int n_jobs, int width, int height, void* stream) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(n_jobs >= 0 && n_jobs < 65536, "mvp_mp4v_reconstruct: %d jobs", n_jobs);
    MVP_REQUIRE(width > 0 && height > 0 && width <= 8192 && height <= 8192, "mvp_mp4v_reconstruct: frame %dx%d",
                width, height);
    if (n_jobs == 0) return MVP_OK;
    MVP_REQUIRE(jobs_dev != nullptr, "mvp_mp4v_reconstruct: NULL jobs");
    ReconParams p{static_cast<const Job*>(jobs_dev), width, height, (width + 15) / 16, (height + 15) / 16};
    hipLaunchKernelGGL(mp4v_recon_kernel, dim3((unsigned)(p.mb_w * p.mb_h), (unsigned)n_jobs), dim3(64), 0,
                       reinterpret_cast<hipStream_t>(stream), p);
    MVP_HIP(hipGetLastError());
    MVP_ABI_END
}
