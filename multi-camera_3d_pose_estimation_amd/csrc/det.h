// Internal (not part of the C-ABI): person-detector kernels (det.hip) used by the
// detector graph runtime (detnet.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace mvp {

// Detector conv weights are padded to whole 32-cout rows ([det_cout_pad(cout)][kh][kw][cin]).
inline int det_cout_pad(int cout) { return (cout + 31) / 32 * 32; }

// mmcv rescale_size for scale (S, S), keep_ratio: the resized extent of an H x W frame.
void det_rescale_size(int H, int W, int S, int& nh, int& nw);
void launch_det_letterbox(const uint8_t* frames, int n, int H, int W, int S, const float* mean3, const float* std3,
                          void* out, hipStream_t s);
// 3x3/s2 conv 4 -> 32 channels on the letterboxed [n][S][S][4] input, w f32 [32][9][4].
void launch_det_stem(const uint16_t* x, const float* w, const float* b, uint16_t* y, int n, int S, int act,
                     hipStream_t s);
// the letterbox folded into the stem: the stem stages its input rows letterboxed from the raw
// [n][H][W][3] uint8 frames (bit-identical to launch_det_letterbox + launch_det_stem)
void launch_det_letterbox_stem(const uint8_t* frames, int H, int W, const float* mean3, const float* std3,
                               const float* w, const float* b, uint16_t* y, int n, int S, int act, hipStream_t s);
void launch_det_dw5(const uint16_t* x, int xs, uint16_t* y, int ys, const float* w, const float* b, int n, int H, int W,
                    int C, int act, hipStream_t s);
// conv (1x1, or 3x3 stride 1 / 2, pad ks/2) as a GEMM over the flat output pixels with the
// im2col gathered by DMA; w [det_cout_pad(N)][ks][ks][cin] bf16; act as ConvLaunch.relu (2 = SiLU
// before the residual, 1 = ReLU after it)
// Producer passes folded into a 1x1 conv's pixel DMA on the persistent GEMM (round 6), the
// producer's own launch skipped: `up` = input channels [0, up_c) are the nearest-2x upsample of
// an H/2 x W/2 plane at up (pixel stride up_s; the neck's DET_UP2); `ca` = [n][cin] f32 scales
// applied to every input channel as it lands (DET_CA's in-place pass).  Bit-identical to running
// the producer.
struct DetConvFold {
    const uint16_t* up = nullptr;
    int up_s = 0, up_c = 0;
    const float* ca = nullptr;
};
// whether a conv of this shape runs on the persistent 1x1 GEMM with folds (`ca`: the scale
// fold, whose tables hold 8 frames per 128-pixel tile); MVPOSE_DET_FOLD=0 turns folding off
bool det_conv_fold_ok(int H, int W, int cin, int N, int ks, bool ca);
void launch_det_conv_gemm(const uint16_t* x, int xs, const uint16_t* w, const float* bias, const uint16_t* res, int rs,
                          uint16_t* y, int ys, int n, int H, int W, int cin, int N, int ks, int stride, int act,
                          hipStream_t s, const uint16_t* wimg = nullptr, const uint16_t* wband = nullptr,
                          int live = 0,  // live: couts with non-zero weights or bias (0 = all N)
                          const DetConvFold* fold = nullptr);
// A CSPNeXtBlock's depthwise 5x5 (dw_w [C/8][25][8] f32, dw_b [C]) and pointwise 1x1 (wimg: the
// GEMM weight image of the [det_cout_pad(N) == C][C] weights, pw_b [C]) in one launch, the
// intermediate kept in LDS; bit-identical to launch_det_dw5 + launch_det_conv_gemm (ks 1).
bool det_dwpw_supported(int C);
void launch_det_dwpw(const uint16_t* x, int xs, const float* dw_w, const float* dw_b, const uint16_t* wimg,
                     const float* pw_b, const uint16_t* res, int rs, uint16_t* y, int ys, int n, int H, int W, int C,
                     int N, int act_dw, int act_pw, hipStream_t s);
// The GEMM kernel's weight image (same element count as w: npad x K, K = ks * ks * cin)
void det_pack_gemm_weights(const uint16_t* w, uint16_t* img, int npad, int K, hipStream_t s);
// The band-halo kernel (3x3/s1, >= 96 input channels, 80x80 / 40x40 planes, couts in blocks of 64):
// whether a conv qualifies, and its weight image (same element count as w)
bool det_band_eligible(int H, int W, int cin, int npad, int ks, int stride);
int det_band_rows(int npad);  // cout rows of the band image (npad rounded up to the 64-cout blocks)
void det_pack_band_weights(const uint16_t* w, uint16_t* img, int npad, int cin, hipStream_t s);
// channel attention in place; scratch: [n][17][C] f32 (per-split partial sums + scales)
void launch_det_ca(uint16_t* x, int xs, int n, int HW, int C, const float* wt, const float* b, float* scratch,
                   hipStream_t s, bool scale_pass = true);
// the [n][C] scales launch_det_ca leaves in its scratch
inline const float* det_ca_scales(const float* scratch, int n, int C) { return scratch + (size_t)n * 16 * C; }
void launch_det_spp(uint16_t* buf, int xs, int n, int H, int W, int C, hipStream_t s);
void launch_det_up2(const uint16_t* x, int xs, uint16_t* y, int ys, int n, int H, int W, int C, hipStream_t s);
void launch_det_head(const uint16_t* x, int xs, int F, const float* w, const float* b, float* cand, int n, int H, int W,
                     int stride, int size, int n_priors, int prior0, hipStream_t s);
void launch_det_select(const float* cand, int n, int n_priors, float score_thr, float fx, float fy, float* best,
                       hipStream_t s);

}  // namespace mvp
