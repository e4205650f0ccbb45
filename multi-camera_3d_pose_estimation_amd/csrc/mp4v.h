// MPEG-4 Part 2 split decode: the host entropy-decodes a VOP into one record per macroblock
// plus a list of inverse-quantised coefficients (mp4v.cpp, parse mode); the device
// reconstructs the picture from them — FFmpeg's simple IDCT, half-pel motion compensation with
// edge clamping, I420 -> BGR24 — bit-identical to the host decoder's own reconstruction
// (mp4v_recon.hip).  Layouts shared by both sides and documented in include/mvpose.h.
#pragma once
#include <cstdint>

namespace mp4v {

enum : uint8_t {
    MB_INTRA = 0,  // the six blocks' IDCT put (no prediction)
    MB_INTER = 1,  // motion-compensated prediction (4 luma vectors, 1 chroma) + IDCT residual
    MB_COPY = 2,   // not coded: the reference macroblock (= inter, vectors 0, no residual)
    MB_LOST = 3,   // not reached (a video packet skipped it): the picture buffer is left as it is
};

struct MbRec {             // 32 B, one per macroblock of a parsed VOP, raster order
    uint8_t kind;
    uint8_t nnz[6];        // coefficient entries of each block (0..64)
    uint8_t pad0;
    int16_t mv[4][2];      // luma 8x8 block vectors (half-pel)
    int16_t cmv[2];        // chroma vector (half-pel)
    uint32_t coef;         // the MB's first entry in the VOP's coefficient list
};
static_assert(sizeof(MbRec) == 32, "MbRec is 32 bytes");

// coefficient entry: raster position (0..63) << 16 | (uint16) inverse-quantised value
inline uint32_t coef_entry(int pos, int value) { return (uint32_t)pos << 16 | (uint16_t)(int16_t)value; }

struct Job {               // 48 B: one VOP of one stream slot
    const MbRec* rec;
    const uint32_t* coef;
    uint8_t* cur;          // the picture this VOP writes: Y (16 mb_w x 16 mb_h), then U, V (8 mb_w x 8 mb_h)
    const uint8_t* ref;    // the previous picture (prediction source), same layout
    uint8_t* bgr;          // [height][width][3] output, or NULL (a frame decoded only as a reference)
    int32_t coded;         // 0: not-coded VOP, cur is output again unchanged
    int32_t rounding;      // vop_rounding_type
};
static_assert(sizeof(Job) == 48, "Job is 48 bytes");

}  // namespace mp4v
