// Shared device helpers of the 32x32x16-MFMA convolution kernels (tconv.hip,
// tblock.hip, tblock64.hip): LDS-DMA, epilogue packing, the permuted-cout A rows
// and the bank-conflict-free lane -> pixel maps of a 32-pixel B fragment.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace mvp {
namespace mfma_tile {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

// 16 bytes per lane global -> LDS (M0 + lane*16), no VGPR staging
__device__ __forceinline__ void glds16(const void* src, void* lds_base) {
    __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)lds_base, 16, 0, 0);
}
__device__ __forceinline__ float relu1_asm(float v) {  // one v_max_f32 (fmaxf adds a canonicalize)
    float r;
    asm("v_max_f32 %0, 0, %1" : "=v"(r) : "v"(v));
    return r;
}
// ReLU the compiler can see: the inline-asm form above hides its operand from the hazard
// recognizer, so applied straight to an MFMA result it read the accumulator before the
// MFMA had written it (stem2: couts 16h+0/1 wrong).  __builtin_amdgcn_fmed3f(v, 0, +inf)
// is one v_med3_f32 with the required wait states.
__device__ __forceinline__ float relu1(float v) { return __builtin_amdgcn_fmed3f(v, 0.f, __builtin_inff()); }
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {  // RNE, v_cvt_pk_bf16_f32
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){lo, hi}, bf16x2));
}
__device__ __forceinline__ float lo_bf16(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_bf16(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

// cout held by A row r of a 32-cout group: row 8j+4h+i -> cout 16h+4j+i, so that the
// accumulator lane (column = pixel, k-half h) owns couts 16h .. 16h+15 in order
__host__ __device__ constexpr int row_cout(int r) { return 16 * ((r >> 2) & 1) + 4 * (r >> 3) + (r & 3); }

// ds_read_b128 serves a wave in 4 lane groups of 16 ({0-3,12-15,20-27}, {4-11,16-19,28-31}
// and the same +32); a group is conflict-free when its 16 slots are distinct mod 16.  A
// 32-pixel fragment that wraps an image row shifts the pixels after the wrap by the pad
// slot (2-way conflicts: 43 % extra LDS cycles measured on the 64-ch plane), so lanes
// are mapped to pixels group by group: each lane group reads a row-contiguous 16-pixel
// run.  frag_pixel returns the tile pixel (row-major [crop][row][col]) of fragment f,
// column r32.
__device__ __forceinline__ int lane_rank(int r32, int& g2) {
    if (r32 < 4) { g2 = 0; return r32; }
    if (r32 < 12) { g2 = 1; return r32 - 4; }
    if (r32 < 16) { g2 = 0; return r32 - 8; }
    if (r32 < 20) { g2 = 1; return r32 - 8; }
    if (r32 < 28) { g2 = 0; return r32 - 12; }
    g2 = 1;
    return r32 - 16;
}
template <int W, int TH, int NB>
__device__ __forceinline__ int frag_pixel(int f, int r32) {
    int g2;
    const int rank = lane_rank(r32, g2), g = 2 * f + g2;
    if constexpr (W % 16 == 0) {
        return g * 16 + rank;  // 16-pixel runs never straddle a row
    } else if constexpr (W == 24 && TH == 16 && NB == 1) {
        // 16 head runs (row r, x 0..15), then 8 tail pairs (rows k and k+8, x 16..23):
        // 8 rows of pitch 25 slots = 200 = 8 mod 16, so the two halves use disjoint banks
        if (g < 16) return g * 24 + rank;
        const int k = g - 16;
        return rank < 8 ? k * 24 + 16 + rank : (k + 8) * 24 + 8 + rank;
    } else {
        return f * 32 + r32;
    }
}

// 8x4 pixel blocks (images of W % 4 == 0 at a row pitch RS = 2 mod 4, e.g. W + 2 slots with
// a zero pad on each side): lane r32 -> (row, col) of the block, block b = r32 / 4 of 4 lanes;
// lane group {0-3,12-15,20-27} (b = 0, 3, 5, 6) takes rows 0, 2, 4, 6 and {4-11,16-19,28-31}
// (b = 1, 2, 4, 7) rows 1, 3, 5, 7.  Row i starts at residue i * RS mod 16 = multiples of 4
// (even rows) and of 4 plus 2 (odd rows), distinct within a group, so every tap's 16 slots
// per group are distinct mod 16 — conflict-free ds_read_b128 with any constant tap offset.
// grp = the lane group, pos = rank within it (0-15): 2 x 16 blocks use (grp, pos).
__device__ __forceinline__ int lane_grp(int r32) { return (0x96 >> (r32 >> 2)) & 1; }
__device__ __forceinline__ int lane_pos(int r32) { return 4 * (r32 >> 3) + (r32 & 3); }
__device__ __forceinline__ int blk_row(int r32) { return 2 * (r32 >> 3) + lane_grp(r32); }
__device__ __forceinline__ int blk_col(int r32) { return r32 & 3; }

// Tile pixel (row-major [crop][row][col]) of fragment f on 8x4 blocks: per crop TH/8 x W/4
// blocks, row-block-major.
template <int W, int TH, int NB>
__device__ __forceinline__ int frag_pixel_blk(int f, int r32) {
    static_assert(W % 4 == 0 && TH % 8 == 0, "8x4 blocks");
    constexpr int FC = W / 4, FPC = (TH / 8) * FC;
    const int nb = f / FPC, rem = f - nb * FPC, rb = rem / FC, cb = rem - rb * FC;
    return (nb * TH + 8 * rb + blk_row(r32)) * W + 4 * cb + blk_col(r32);
}

}  // namespace mfma_tile
}  // namespace mvp
