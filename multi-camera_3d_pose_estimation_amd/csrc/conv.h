// Internal (not part of the C-ABI): convolution / fuse launchers used by the
// HRNet graph runtime (hrnet.cpp).
#pragma once
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <cstdint>

namespace mvp {

// One NHWC bf16 convolution with BN folded into (w, bias):
//   y = act( conv(x, w) + bias [+ res] )
// w: [Cout_pad][KS][KS][Cin] bf16 (Cout_pad = Cout rounded up to the tile),
// bias: [Cout_pad] f32.  out_f32_nchw: write f32 [N][Cout][Ho][Wo] instead of
// bf16 NHWC (HeatmapHead output).
struct ConvLaunch {
    const uint16_t* x;
    const uint16_t* w;
    const float* bias;
    const uint16_t* res;  // nullable, same shape as y
    uint16_t* y;          // bf16 NHWC [N][Ho][Wo][Cout]
    float* yf;            // f32 NCHW (when out_f32_nchw)
    int N, H, W, Cin, Cout;
    int ks, stride, relu, out_f32_nchw;
    // 1x1 only: second input (graph cat-fusion) — channels [c1, Cin) of the conv come
    // from x2 [N][H][W][Cin - c1], the first c1 from x
    const uint16_t* x2 = nullptr;
    int c1 = 0;
    // Channel views (detector graph, detnet.cpp): elements between consecutive pixels of
    // x / y / res when they are channel slices of wider NHWC tensors (0 = dense: Cin /
    // Cout).  relu == 2 selects SiLU (x * sigmoid(x)) applied BEFORE the residual add
    // (CSPNeXtBlock: conv2(conv1(x)) + x); ReLU (1) is applied after it.
    int x_stride = 0, y_stride = 0, r_stride = 0;
    // w re-laid as tconv16's weight image (tconv16_pack_weights) when the graph made one: the
    // 128/256-channel branch planes then run tconv16.hip (nullptr: tconv.hip), and s2conv's
    // streamed-weight planes read it instead of w
    const uint16_t* w_img = nullptr;
};

void launch_conv(const ConvLaunch& c, hipStream_t s);
// The generic implicit-GEMM conv (conv_mfma_kernel) only, with channel views and the
// SiLU epilogue: no HRNet-plane kernel is tried.  bf16 NHWC output.
void launch_conv_generic(const ConvLaunch& c, hipStream_t s);

// Heatmap head (conv1x1.hip): 1x1 32 -> 17 + bias, f32 NCHW output; false otherwise
// (or MVPOSE_NO_HEAD1X1=1).
bool launch_head1x1(const ConvLaunch& c, hipStream_t s);
// The head with the last fuse layer folded in (graph pass head_fuse, conv1x1.hip): in[k]
// bf16 NHWC [N][H/up_k][W/up_k][32] summed (nearest upsample), optional ReLU, rounded to
// bf16 (out0 exactly as launch_fuse_sum writes it), then 1x1 32 -> 17 + bias, f32 NCHW y.
bool head_fuse_supported(int cin, int cout, int n_in);
void launch_head_fuse(const uint16_t* const* in, const int* up, int n_in, int relu, const uint16_t* w,
                      const float* bias, float* y, int N, int H, int W, hipStream_t s);

// Direct-load 1x1 conv (conv1x1.hip); false when the conv is not a bf16-output 1x1.
bool launch_conv1x1_direct(const ConvLaunch& c, hipStream_t s);

// Bottleneck join (conv1x1.hip): y = relu(W1·[x | x2] + b1 [+ res]) with 256 couts,
// then y2 = relu(W2·y + b2) with 64 couts from the bf16 y still in registers (the
// next Bottleneck's conv1), so y is written once and never re-read for it.
// W1 [256][cin1 (+ cin2)] bf16, W2 [64][256] bf16.  cin1 + cin2 must be 64 or 128.
struct PairLaunch {
    const uint16_t* x = nullptr;
    const uint16_t* x2 = nullptr;  // dual input (cat-fused downsample) or nullptr
    int c1 = 0, c2 = 0;            // channels of x, x2
    const uint16_t* w1 = nullptr;
    const float* b1 = nullptr;
    const uint16_t* res = nullptr;  // 256-ch residual or nullptr
    uint16_t* y = nullptr;
    const uint16_t* w2 = nullptr;
    const float* b2 = nullptr;
    uint16_t* y2 = nullptr;
    long n_pix = 0;
};
bool conv1x1_pair_supported(int cin_total, int cmid, int cout2);
void launch_conv1x1_pair(const PairLaunch& p, hipStream_t s);


// Streaming fused Bottleneck on layer1's 256-ch 64x48 plane (bneck.hip): y = relu(W3 ·
// relu(conv3x3(relu(W1 · x + b1), W2) + b2) + b3 + x), W1 [64][256], W2 [64][3][3][64], W3
// [256][64] bf16; the two 64-ch intermediates never leave LDS.  perm selects conv1's K order:
// the Bottleneck join's (conv1x1_pair second GEMM, 1) or the plain 1x1 kernel's (0), so the
// result is bit-identical to the unfused graph either way.  bneck_supported is false for
// other shapes (or MVPOSE_NO_BNECK=1).
struct BneckLaunch {
    const uint16_t* x = nullptr;
    const uint16_t* w1 = nullptr;
    const float* b1 = nullptr;
    const uint16_t* w2 = nullptr;
    const float* b2 = nullptr;
    const uint16_t* w3 = nullptr;
    const float* b3 = nullptr;
    uint16_t* y = nullptr;
    int N = 0, H = 0, W = 0;
    int perm = 1;
    // layer1's first block: x has 64 channels, w3 / b3 are the cat-fused [conv3 | downsample]
    // weights [256][128] and summed biases (no residual)
    int lead = 0;
    // y in chunk-planar layout [N][16][64][48][16] (16-channel chunks; the graph sets it when y
    // feeds only trans1, which then reads it planar)
    int planar = 0;
};
bool bneck_supported(int H, int W, int C, int M);
void launch_bneck(const BneckLaunch& c, hipStream_t s);

// Lean 3x3/s1 conv on 32x32x16 MFMAs for 384-pixel x 64-cout tiles (tconv.hip):
// 64 ch @ 32x24 and 64x48, 128 ch @ 16x12, 256 ch @ 8x6 (ReLU epilogue).  false
// when the conv is not one of those (or MVPOSE_NO_TCONV=1).
bool launch_tconv(const ConvLaunch& c, hipStream_t s);
// 128-cout-tile version for 128 ch @ 16x12 and 256 ch @ 8x6 (tconv16.hip), tried first by
// launch_tconv; false otherwise (no weight image, or MVPOSE_TCONV16=0).
bool launch_tconv16(const ConvLaunch& c, hipStream_t s);
// Elements of the weight image of a conv tconv16 serves (0: not one of its planes), and the
// packing launch (w [cout][3][3][cin] -> img, same element count).
long tconv16_image_elems(int cin, int cout, int h, int w, int ks, int stride);
void tconv16_pack_weights(const uint16_t* w, uint16_t* img, int cin, int cout, hipStream_t s);

// 3x3/s2 conv on a polyphase halo, 16-channel items (s2conv.hip): transitions 2/3
// and the downsampling fuse-layer convs of HRNet-W32 with >= 64 couts (no residual).
// false when the conv is not one of those planes (or MVPOSE_NO_S2CONV=1).
bool launch_s2conv(const ConvLaunch& c, hipStream_t s);

// Sibling 3x3/s2 convs on one input (graph sib-fusion, s2conv.hip): up to 3 outputs whose
// weights are concatenated along cout (w [128][3][3][Cin], zero rows past the last
// output; bias [128]); output i gets couts [sum_{j<i} cout_j, + cout_i) with its own ReLU.
struct S2Multi {
    const uint16_t* x = nullptr;
    const uint16_t* w = nullptr;
    const float* bias = nullptr;
    int N = 0, H = 0, W = 0, Cin = 0;
    int n_out = 0;
    uint16_t* y[3] = {nullptr, nullptr, nullptr};
    int cout[3] = {0, 0, 0};
    int relu[3] = {0, 0, 0};
};
bool s2conv_multi_supported(int H, int W, int Cin, int total_cout);
void launch_s2conv_multi(const S2Multi& m, hipStream_t s);

// 3x3/s2 stem conv on 4-channel (RGB + zero) bf16 crops, BN folded, ReLU.
// w: [64][3][3][4] f32, bias [64] f32.  x [N][H][W][4] -> y [N][H/2][W/2][64].
void launch_stem(const uint16_t* x, const float* w, const float* bias, uint16_t* y, int N, int H, int W,
                 hipStream_t s);

// Fused stem (stem2.hip): conv1 (3x3/s2 4 -> 64, w1 f32 [64][3][3][4]) and conv2 (3x3/s2
// 64 -> 64, w2 bf16 [64][3][3][64]), both BN-folded with ReLU, in one launch; conv1's
// output never leaves LDS.  x [N][256][192][4] -> y [N][64][48][64].  stem2_supported is
// false for other shapes (or MVPOSE_NO_STEMFUSE=1).
// Crop-streaming kernels (tblock32s, tblock64's row reuse, streaming stem2) give each workgroup
// a contiguous crop range: worth it only when every CU gets at least one crop; below that the
// caller takes the per-tile kernel, which spreads N * tiles-per-crop items over every CU.
// (Measured, profiles/r04_crop_ranges_ab.txt: the tile kernels win 22 % at 40 crops and 1.8 % at
// 160; at 400 crops -- ragged 1-2 crops per CU -- the crop ranges still win, row reuse included.)
inline bool crop_ranges_balanced(int N, int cus) {
    const char* e = getenv("MVPOSE_CROP_STREAM");  // tests: 1 = the crop-streaming kernels at any batch
    if (e && e[0] == '1') return true;
    return N >= cus;
}
bool stem2_supported(int H, int W, int cin2, int cout2);
void launch_stem2(const uint16_t* x, const float* w1, const float* b1, const uint16_t* w2, const float* b2,
                  uint16_t* y, int N, int H, int W, hipStream_t s);

// Transition1 (trans1.hip): t0 = relu(conv3x3/s1(x, w0) + b0) (256 -> 32) and t1 =
// relu(conv3x3/s2(x, w1) + b1) (256 -> 64) from ONE pass over x [N][64][48][256];
// w0 [32][3][3][256] and w1 [64][3][3][256] bf16 at element offsets w0_off / w1_off of wb.  trans1_supported is false for other
// shapes (or MVPOSE_NO_TRANSFUSE=1).
bool trans1_supported(int H, int W, int C, int cout0, int cout1);
void launch_trans1(const uint16_t* x, const uint16_t* wb, int64_t w0_off, const float* b0, int64_t w1_off,
                   const float* b1, uint16_t* y0, uint16_t* y1, int N, hipStream_t s,
                   const uint16_t* wimg = nullptr, bool planar = false);
// trans1's weight image (9 x 2 x 96 16-B slots per 16-channel chunk, 221,184 elements)
constexpr long kTrans1ImageElems = 16L * 9 * 2 * 96 * 8;
void trans1_pack_weights(const uint16_t* wb, int64_t w0_off, int64_t w1_off, uint16_t* img, hipStream_t s);

// HRModule fuse: out = relu( sum_i up_i(in_i) ), nearest upsample factor up_i
// (1, 2, 4, 8); all tensors bf16 NHWC with C channels, out at resolution H x W.
void launch_fuse_sum(const uint16_t* const* in, const int* up, int n_in, uint16_t* out, int N, int H, int W,
                     int C, int relu, hipStream_t s);

// Conv weight padding rule shared with the host packer.
int conv_cout_pad(int cout);

// 64 KiB of device zeros (out-of-image DMA source), allocated on first use.
const uint16_t* conv_zero_region();

// Fused BasicBlock on 32 channels (block.hip):
//   y = relu(conv3x3(relu(conv3x3(x, w1) + b1), w2) + b2 + x), all bf16 NHWC [N][H][W][32],
// w1/w2 [32][3][3][32] bf16, b1/b2 [32] f32.  Bit-identical to the two convs run separately.
bool basic_block_c32_supported(int H, int W);
// 32x32x16 version of the fused block (tblock.hip) for W = 48, H % 16 == 0; false when
// not applicable (or MVPOSE_NO_TBLOCK=1).  Not bit-identical to the separate convs.
bool launch_tblock32s(const uint16_t* x, const uint16_t* w1, const float* b1, const uint16_t* w2, const float* b2,
                      uint16_t* y, int N, int H, int W, hipStream_t s);
bool launch_tblock32(const uint16_t* x, const uint16_t* w1, const float* b1, const uint16_t* w2, const float* b2,
                     uint16_t* y, int N, int H, int W, hipStream_t s);
void launch_basic_block_c32(const uint16_t* x, const uint16_t* w1, const float* b1, const uint16_t* w2,
                            const float* b2, uint16_t* y, int N, int H, int W, hipStream_t s);
// The same block on 64 channels at 32x24 (tblock64.hip, warp-specialised, weights in
// registers); bit-identical to the two tconv launches.  Supported unless MVPOSE_NO_TBLOCK64=1.
bool tblock64_supported(int H, int W);
void launch_tblock64(const uint16_t* x, const uint16_t* w1, const float* b1, const uint16_t* w2, const float* b2,
                     uint16_t* y, int N, int H, int W, hipStream_t s);

}  // namespace mvp
