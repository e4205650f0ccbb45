// MPEG-4 Part 2 (ISO/IEC 14496-2) Simple Profile VLC and scan tables, restated for the
// host-side mp4v decoder (mp4v.cpp).  Codes are (code, length) pairs, MSB first.
//
// The reference reads its recordings with cv.VideoCapture (utils.py:867), i.e. FFmpeg's
// mpeg4 decoder for the 'mp4v' files synchronize_videos.py:64,240 writes; FFmpeg is not in
// this image, so these are restated from the standard's tables (B-6/B-7 MCBPC, B-8 CBPY,
// B-12 MVD, B-13/B-14 DC size, B-16/B-17 TCOEF, 7-1 DC scaler, the zig-zag and alternate
// scans).  mvp_mp4v_selfcheck verifies the properties a transcription error would break:
// every table is prefix-free and complete (Kraft sum 1, with the escape / stuffing codes), the
// intra TCOEF codes are a permutation of the inter ones, the run/level tables follow the
// standard's LMAX order, and the scans are permutations (tests/test_mp4v.py).
#pragma once
#include <cstdint>

namespace mp4v {

struct Code {
    uint16_t code;
    uint8_t len;
};

// Table B-6: MCBPC for I-VOPs.  index = (mb_type == 4 ? 4 : 0) + cbpc; 8 = stuffing.
static const Code kMcbpcIntra[9] = {{1, 1}, {1, 3}, {2, 3}, {3, 3}, {1, 4}, {1, 6}, {2, 6}, {3, 6}, {1, 9}};

// Table B-7: MCBPC for P-VOPs.  index = cbpc | intra << 2 | dquant << 3 | inter4v << 4
// (0-3 inter, 4-7 intra, 8-11 inter+q, 12-15 intra+q, 16-19 inter4v, 20 stuffing, 24-27
// inter4v+q, H.263's extension; 21-23 unused).
static const Code kMcbpcInter[28] = {
    {1, 1},  {3, 4},   {2, 4},   {5, 6},    // inter
    {3, 5},  {4, 8},   {3, 8},   {3, 7},    // intra
    {3, 3},  {7, 7},   {6, 7},   {5, 9},    // inter + q
    {4, 6},  {4, 9},   {3, 9},   {2, 9},    // intra + q
    {2, 3},  {5, 7},   {4, 7},   {5, 8},    // inter4v
    {1, 9},  {0, 0},   {0, 0},   {0, 0},    // stuffing
    {2, 11}, {12, 13}, {14, 13}, {15, 13},  // inter4v + q
};

// Table B-8: CBPY (the intra meaning; inter macroblocks use 15 - value).
static const Code kCbpy[16] = {{3, 4}, {5, 5}, {4, 5}, {9, 4}, {3, 5}, {7, 4}, {2, 6}, {11, 4},
                               {2, 5}, {3, 6}, {5, 4}, {10, 4}, {4, 4}, {8, 4}, {6, 4}, {3, 2}};

// Table B-12: MVD magnitude codes 0..32 (a sign bit follows every non-zero code).
static const Code kMvd[33] = {{1, 1},  {1, 2},  {1, 3},  {1, 4},  {3, 6},  {5, 7},  {4, 7},  {3, 7},  {11, 9},
                              {10, 9}, {9, 9},  {17, 10}, {16, 10}, {15, 10}, {14, 10}, {13, 10}, {12, 10},
                              {11, 10}, {10, 10}, {9, 10}, {8, 10}, {7, 10}, {6, 10}, {5, 10}, {4, 10},
                              {7, 11}, {6, 11}, {5, 11}, {4, 11}, {3, 11}, {2, 11}, {3, 12}, {2, 12}};

// Tables B-13 / B-14: dct_dc_size for luminance / chrominance, sizes 0..12.
static const Code kDcLum[13] = {{3, 3}, {3, 2}, {2, 2}, {2, 3}, {1, 3},  {1, 4}, {1, 5},
                                {1, 6}, {1, 7}, {1, 8}, {1, 9}, {1, 10}, {1, 11}};
static const Code kDcChrom[13] = {{3, 2}, {2, 2}, {1, 2}, {1, 3},  {1, 4},  {1, 5}, {1, 6},
                                  {1, 7}, {1, 8}, {1, 9}, {1, 10}, {1, 11}, {1, 12}};

// Tables B-16 (intra) / B-17 (inter): TCOEF events in (last, run, level) order, escape last.
constexpr int kTcoefEvents = 102;
constexpr int kTcoefNotLastIntra = 67, kTcoefNotLastInter = 58;

static const Code kTcoefIntra[kTcoefEvents + 1] = {
    {0x2, 2},   {0x6, 3},   {0xf, 4},   {0xd, 5},   {0xc, 5},   {0x15, 6},  {0x13, 6},  {0x12, 6},
    {0x17, 7},  {0x1f, 8},  {0x1e, 8},  {0x1d, 8},  {0x25, 9},  {0x24, 9},  {0x23, 9},  {0x21, 9},
    {0x21, 10}, {0x20, 10}, {0xf, 10},  {0xe, 10},  {0x7, 11},  {0x6, 11},  {0x20, 11}, {0x21, 11},
    {0x50, 12}, {0x51, 12}, {0x52, 12}, {0xe, 4},   {0x14, 6},  {0x16, 7},  {0x1c, 8},  {0x20, 9},
    {0x1f, 9},  {0xd, 10},  {0x22, 11}, {0x53, 12}, {0x55, 12}, {0xb, 5},   {0x15, 7},  {0x1e, 9},
    {0xc, 10},  {0x56, 12}, {0x11, 6},  {0x1b, 8},  {0x1d, 9},  {0xb, 10},  {0x10, 6},  {0x22, 9},
    {0xa, 10},  {0xd, 6},   {0x1c, 9},  {0x8, 10},  {0x12, 7},  {0x1b, 9},  {0x54, 12}, {0x14, 7},
    {0x1a, 9},  {0x57, 12}, {0x19, 8},  {0x9, 10},  {0x18, 8},  {0x23, 11}, {0x17, 8},  {0x19, 9},
    {0x18, 9},  {0x7, 10},  {0x58, 12}, {0x7, 4},   {0xc, 6},   {0x16, 8},  {0x17, 9},  {0x6, 10},
    {0x5, 11},  {0x4, 11},  {0x59, 12}, {0xf, 6},   {0x16, 9},  {0x5, 10},  {0xe, 6},   {0x4, 10},
    {0x11, 7},  {0x24, 11}, {0x10, 7},  {0x25, 11}, {0x13, 7},  {0x5a, 12}, {0x15, 8},  {0x5b, 12},
    {0x14, 8},  {0x13, 8},  {0x1a, 8},  {0x15, 9},  {0x14, 9},  {0x13, 9},  {0x12, 9},  {0x11, 9},
    {0x26, 11}, {0x27, 11}, {0x5c, 12}, {0x5d, 12}, {0x5e, 12}, {0x5f, 12}, {0x3, 7},
};

static const int8_t kRunIntra[kTcoefEvents] = {
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
    0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 5,
    6, 6, 6, 7, 7, 7, 8, 8, 9, 9, 10, 11, 12, 13, 14, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1,
    2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20,
};
static const int8_t kLevelIntra[kTcoefEvents] = {
    1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26,
    27, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 1, 2, 3, 4, 5, 1, 2, 3, 4, 1, 2, 3, 1, 2, 3,
    1, 2, 3, 1, 2, 3, 1, 2, 1, 2, 1, 1, 1, 1, 1, 1, 2, 3, 4, 5, 6, 7, 8, 1, 2, 3,
    1, 2, 1, 2, 1, 2, 1, 2, 1, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
};

static const Code kTcoefInter[kTcoefEvents + 1] = {
    {0x2, 2},   {0xf, 4},   {0x15, 6},  {0x17, 7},  {0x1f, 8},  {0x25, 9},  {0x24, 9},  {0x21, 10},
    {0x20, 10}, {0x7, 11},  {0x6, 11},  {0x20, 11}, {0x6, 3},   {0x14, 6},  {0x1e, 8},  {0xf, 10},
    {0x21, 11}, {0x50, 12}, {0xe, 4},   {0x1d, 8},  {0xe, 10},  {0x51, 12}, {0xd, 5},   {0x23, 9},
    {0xd, 10},  {0xc, 5},   {0x22, 9},  {0x52, 12}, {0xb, 5},   {0xc, 10},  {0x53, 12}, {0x13, 6},
    {0xb, 10},  {0x54, 12}, {0x12, 6},  {0xa, 10},  {0x11, 6},  {0x9, 10},  {0x10, 6},  {0x8, 10},
    {0x16, 7},  {0x55, 12}, {0x15, 7},  {0x14, 7},  {0x1c, 8},  {0x1b, 8},  {0x21, 9},  {0x20, 9},
    {0x1f, 9},  {0x1e, 9},  {0x1d, 9},  {0x1c, 9},  {0x1b, 9},  {0x1a, 9},  {0x22, 11}, {0x23, 11},
    {0x56, 12}, {0x57, 12}, {0x7, 4},   {0x19, 9},  {0x5, 11},  {0xf, 6},   {0x4, 11},  {0xe, 6},
    {0xd, 6},   {0xc, 6},   {0x13, 7},  {0x12, 7},  {0x11, 7},  {0x10, 7},  {0x1a, 8},  {0x19, 8},
    {0x18, 8},  {0x17, 8},  {0x16, 8},  {0x15, 8},  {0x14, 8},  {0x13, 8},  {0x18, 9},  {0x17, 9},
    {0x16, 9},  {0x15, 9},  {0x14, 9},  {0x13, 9},  {0x12, 9},  {0x11, 9},  {0x7, 10},  {0x6, 10},
    {0x5, 10},  {0x4, 10},  {0x24, 11}, {0x25, 11}, {0x26, 11}, {0x27, 11}, {0x58, 12}, {0x59, 12},
    {0x5a, 12}, {0x5b, 12}, {0x5c, 12}, {0x5d, 12}, {0x5e, 12}, {0x5f, 12}, {0x3, 7},
};

static const int8_t kRunInter[kTcoefEvents] = {
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 4,
    4, 4, 5, 5, 5, 6, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20,
    21, 22, 23, 24, 25, 26, 0, 0, 0, 1, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16,
    17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38, 39, 40,
};
static const int8_t kLevelInter[kTcoefEvents] = {
    1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 1, 2, 3, 4, 5, 6, 1, 2, 3, 4, 1, 2, 3, 1,
    2, 3, 1, 2, 3, 1, 2, 3, 1, 2, 1, 2, 1, 2, 1, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
    1, 1, 1, 1, 1, 1, 1, 2, 3, 1, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
    1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
};

// Zig-zag and the alternate horizontal scan (raster index 8 * row + column); the alternate
// vertical scan is the horizontal one transposed.
static const uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
static const uint8_t kAltHorizontal[64] = {0,  1,  2,  3,  8,  9,  16, 17, 10, 11, 4,  5,  6,  7,  15, 14,
                                           13, 12, 19, 18, 24, 25, 32, 33, 26, 27, 20, 21, 22, 23, 28, 29,
                                           30, 31, 34, 35, 40, 41, 48, 49, 42, 43, 36, 37, 38, 39, 44, 45,
                                           46, 47, 50, 51, 56, 57, 58, 59, 52, 53, 54, 55, 60, 61, 62, 63};

// Default quantisation matrices of quant_type 1 (MPEG), raster order.
static const uint8_t kDefaultIntraMatrix[64] = {
    8,  17, 18, 19, 21, 23, 25, 27, 17, 18, 19, 21, 23, 25, 27, 28, 20, 21, 22, 23, 24, 26, 28, 30,
    21, 22, 23, 24, 26, 28, 30, 32, 22, 23, 24, 26, 28, 30, 32, 35, 23, 24, 26, 28, 30, 32, 35, 38,
    25, 26, 28, 30, 32, 35, 38, 41, 27, 28, 30, 32, 35, 38, 41, 45};
static const uint8_t kDefaultInterMatrix[64] = {
    16, 17, 18, 19, 20, 21, 22, 23, 17, 18, 19, 20, 21, 22, 23, 24, 18, 19, 20, 21, 22, 23, 24, 25,
    19, 20, 21, 22, 23, 24, 26, 27, 20, 21, 22, 23, 25, 26, 27, 28, 21, 22, 23, 24, 26, 27, 28, 30,
    22, 23, 24, 26, 27, 28, 30, 31, 23, 24, 25, 27, 28, 30, 31, 33};

// intra_dc_vlc_thr -> the QP below which intra DC uses the dct_dc_size VLC (99: always).
static const int kDcThreshold[8] = {99, 13, 15, 17, 19, 21, 23, 0};

}  // namespace mp4v
