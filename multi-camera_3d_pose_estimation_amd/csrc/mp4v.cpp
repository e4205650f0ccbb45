// Host-side MPEG-4 Part 2 Simple Profile video decoder (the 'mp4v' recordings the reference
// writes with cv2.VideoWriter_fourcc(*'mp4v'), synchronize_videos.py:64,240, and reads back
// with cv.VideoCapture in utils.py:849-909 frame_generator / read_video_as_frames).
//
// This image has no codec library (no FFmpeg, cv2, PyAV, rocDecode), so the bitstream is
// decoded here, following ISO/IEC 14496-2 and the choices FFmpeg's mpeg4 decoder makes where the
// standard leaves room (which cv.VideoCapture uses):
//   * VOS / VO / VOL headers (rectangular shape, progressive, 8-bit, no sprites, no data
//     partitioning, no quarter-pel), GOV headers, video packets (resync markers);
//   * I- and P-VOPs, not-coded VOPs (the previous frame again); B- and S-VOPs are rejected;
//   * macroblocks: intra / intra+q, inter / inter+q / inter4v (/ inter4v+q), not-coded;
//   * intra DC by dct_dc_size VLC or in the AC VLC (intra_dc_vlc_thr), DC / AC prediction with
//     FFmpeg's packet-boundary rules, alternate scans, TCOEF escapes (3 types);
//   * H.263 (quant_type 0) and MPEG (quant_type 1, default or loaded matrices) inverse quantisation;
//   * FFmpeg's "simple" integer IDCT (the decoder's default IDCT on x86, bit-exact across its
//     C / SIMD versions): rows then columns, W1..W7 = 22725, 21407, 19266, 16383, 12873, 8867,
//     4520, ROW_SHIFT 11, COL_SHIFT 20, the DC-only row shortcut;
//   * half-pel motion compensation with vop_rounding_type, edge clamping (unrestricted MVs),
//     1MV / 4MV chroma vector rounding, median MV prediction with the first-row rules;
//   * I420 -> BGR24 with BT.601 limited-range integer coefficients (cv2's sws_scale path is
//     table-driven with its own rounding: colour conversion parity is unpinned).
// Parity against cv2 / FFmpeg is UNPINNED (neither exists here; the reference holds no video
// fixture); tests/test_mp4v.py checks the decoder against bitstreams built from known
// coefficients and motion vectors and a numpy restatement of inverse quantisation, IDCT and
// motion compensation.
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "mp4v.h"
#include "mp4v_tables.h"
#include "mvp_common.h"

namespace mp4v {

// ------------------------------------------------------------------ bits and VLCs
struct Bits {
    const uint8_t* p = nullptr;
    size_t n = 0;      // bytes
    size_t pos = 0;    // bits read
    uint32_t show(int k) const {  // 1 <= k <= 25; zero bits past the end
        const size_t byte = pos >> 3;
        uint64_t v;
        if (byte + 8 <= n) {
            std::memcpy(&v, p + byte, 8);
            v = __builtin_bswap64(v);
        } else {
            v = 0;
            for (int i = 0; i < 8; i++) v = (v << 8) | (byte + i < n ? p[byte + i] : 0);
        }
        return (uint32_t)((v << (pos & 7)) >> (64 - k));
    }
    void skip(int k) { pos += k; }
    uint32_t get(int k) {
        if (k == 0) return 0;
        const uint32_t v = show(k);
        pos += k;
        return v;
    }
    int get1() { return (int)get(1); }
    int get_sbits(int k) {  // two's complement
        const int v = (int)get(k);
        return v >= (1 << (k - 1)) ? v - (1 << k) : v;
    }
    int get_xbits(int k) {  // MPEG "dct_dc_differential": MSB 0 = negative
        const int v = (int)get(k);
        return (v >> (k - 1)) ? v : v - ((1 << k) - 1);
    }
    int64_t left() const { return (int64_t)n * 8 - (int64_t)pos; }
    void align() { pos = (pos + 7) & ~(size_t)7; }
};

struct Vlc {
    int maxlen = 0;
    std::vector<int16_t> sym;
    std::vector<uint8_t> len;
    void build(const Code* codes, int count) {
        maxlen = 0;
        for (int i = 0; i < count; i++) maxlen = std::max(maxlen, (int)codes[i].len);
        sym.assign((size_t)1 << maxlen, -1);
        len.assign((size_t)1 << maxlen, 0);
        for (int i = 0; i < count; i++) {
            if (codes[i].len == 0) continue;
            const int sh = maxlen - codes[i].len;
            const uint32_t base = (uint32_t)codes[i].code << sh;
            for (uint32_t j = 0; j < (1u << sh); j++) {
                sym[base + j] = (int16_t)i;
                len[base + j] = codes[i].len;
            }
        }
    }
    int decode(Bits& b) const {
        const uint32_t v = b.show(maxlen);
        const int s = sym[v];
        if (s >= 0) b.skip(len[v]);
        return s;
    }
};

struct Tables {
    Vlc mcbpc_i, mcbpc_p, cbpy, mvd, dc_lum, dc_chrom, tc_intra, tc_inter;
    // LMAX[last][run], RMAX[last][level] of each TCOEF table (escape types 1 and 2)
    int lmax[2][2][64], rmax[2][2][64];  // [intra][last][...]
    uint8_t scan_zz[64], scan_h[64], scan_v[64];
    Tables() {
        mcbpc_i.build(kMcbpcIntra, 9);
        mcbpc_p.build(kMcbpcInter, 28);
        cbpy.build(kCbpy, 16);
        mvd.build(kMvd, 33);
        dc_lum.build(kDcLum, 13);
        dc_chrom.build(kDcChrom, 13);
        tc_intra.build(kTcoefIntra, kTcoefEvents + 1);
        tc_inter.build(kTcoefInter, kTcoefEvents + 1);
        std::memset(lmax, 0, sizeof(lmax));
        std::memset(rmax, 0, sizeof(rmax));
        for (int t = 0; t < 2; t++) {
            const int8_t* run = t ? kRunIntra : kRunInter;
            const int8_t* lev = t ? kLevelIntra : kLevelInter;
            const int nl = t ? kTcoefNotLastIntra : kTcoefNotLastInter;
            for (int i = 0; i < kTcoefEvents; i++) {
                const int last = i >= nl;
                lmax[t][last][run[i]] = std::max(lmax[t][last][run[i]], (int)lev[i]);
                rmax[t][last][lev[i]] = std::max(rmax[t][last][lev[i]], (int)run[i]);
            }
        }
        for (int i = 0; i < 64; i++) {
            scan_zz[i] = kZigzag[i];
            scan_h[i] = kAltHorizontal[i];
            scan_v[i] = (uint8_t)((kAltHorizontal[i] & 7) * 8 + (kAltHorizontal[i] >> 3));
        }
    }
};

const Tables& tables() {
    static const Tables t;
    return t;
}

// ------------------------------------------------------------------ IDCT (FFmpeg simple IDCT)
constexpr int W1 = 22725, W2 = 21407, W3 = 19266, W4 = 16383, W5 = 12873, W6 = 8867, W7 = 4520;
constexpr int ROW_SHIFT = 11, COL_SHIFT = 20;

inline void idct_row(int16_t* r) {
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

inline void idct_col(const int16_t* c, int (&o)[8]) {
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

inline uint8_t clip8(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

// block: 64 coefficients, raster (8 * row + column); ADD = add to dst instead of put.  When the
// row pass leaves only row 0 non-zero (DC-only and first-row-only blocks, most of a real frame)
// every column reduces to its c[0] term, which is what the full column pass computes for it.
template <bool ADD>
void idct_write_t(int16_t* blk, uint8_t* dst, int stride) {
    int rows = 0;
    for (int r = 0; r < 8; r++) {
        int16_t* q = blk + 8 * r;
        if (r && !(q[0] | q[1] | q[2] | q[3] | q[4] | q[5] | q[6] | q[7])) continue;
        idct_row(q);
        rows |= 1 << r;
    }
    if (rows <= 1) {
        for (int c = 0; c < 8; c++) {
            const int o = (W4 * (blk[c] + ((1 << (COL_SHIFT - 1)) / W4))) >> COL_SHIFT;
            for (int r = 0; r < 8; r++) {
                uint8_t& d = dst[r * stride + c];
                d = clip8(ADD ? d + o : o);
            }
        }
        return;
    }
    for (int c = 0; c < 8; c++) {
        int o[8];
        idct_col(blk + c, o);
        for (int r = 0; r < 8; r++) {
            uint8_t& d = dst[r * stride + c];
            d = clip8(ADD ? d + o[r] : o[r]);
        }
    }
}

void idct_write(int16_t* blk, uint8_t* dst, int stride, bool add) {
    if (add) idct_write_t<true>(blk, dst, stride);
    else idct_write_t<false>(blk, dst, stride);
}

// BT.601 limited range in 8-bit fixed point (y = 298 (Y - 16) + 128, then >> 8 after the chroma
// terms): per row, the chroma terms of each 2 x 2 luma quad are spread to the row's columns,
// B, G and R are formed as three planar rows (plain integer loops the compiler vectorises) and
// interleaved into BGR24.  One body, compiled twice: for the baseline ISA and for AVX2 (picked
// at run time), whose 32-bit min / max the vectoriser needs.
#define MP4V_BGR_ROWS_BODY                                                                        \
    std::vector<int32_t> tb(width), tg(width), tr(width);                                         \
    std::vector<uint8_t> pb(width), pg(width), pr(width);                                         \
    for (int y = 0; y < height; y++) {                                                            \
        const uint8_t* Y = Yp + (size_t)y * ys;                                                   \
        uint8_t* o = out + (size_t)y * width * 3;                                                 \
        if (!(y & 1)) {                                                                           \
            const uint8_t* U = Up + (size_t)(y >> 1) * cs;                                        \
            const uint8_t* V = Vp + (size_t)(y >> 1) * cs;                                        \
            for (int x = 0; x < width; x++) {                                                     \
                const int u = U[x >> 1] - 128, v = V[x >> 1] - 128;                               \
                tb[x] = 516 * u + 128 - 298 * 16;                                                 \
                tg[x] = -100 * u - 208 * v + 128 - 298 * 16;                                      \
                tr[x] = 409 * v + 128 - 298 * 16;                                                 \
            }                                                                                     \
        }                                                                                         \
        const int32_t* __restrict__ cb = tb.data();                                               \
        const int32_t* __restrict__ cg = tg.data();                                               \
        const int32_t* __restrict__ cr = tr.data();                                               \
        uint8_t* __restrict__ ob = pb.data();                                                     \
        uint8_t* __restrict__ og = pg.data();                                                     \
        uint8_t* __restrict__ orr = pr.data();                                                    \
        for (int x = 0; x < width; x++) {                                                         \
            const int c = 298 * Y[x];                                                             \
            ob[x] = (uint8_t)std::min(std::max((c + cb[x]) >> 8, 0), 255);                        \
            og[x] = (uint8_t)std::min(std::max((c + cg[x]) >> 8, 0), 255);                        \
            orr[x] = (uint8_t)std::min(std::max((c + cr[x]) >> 8, 0), 255);                       \
        }                                                                                         \
        for (int x = 0; x < width; x++) {                                                         \
            o[3 * x + 0] = ob[x];                                                                 \
            o[3 * x + 1] = og[x];                                                                 \
            o[3 * x + 2] = orr[x];                                                                \
        }                                                                                         \
    }

void bgr_rows_plain(const uint8_t* Yp, const uint8_t* Up, const uint8_t* Vp, int ys, int cs, int width, int height,
                    uint8_t* out) {
    MP4V_BGR_ROWS_BODY
}

__attribute__((target("avx2"))) void bgr_rows_x86avx2(const uint8_t* Yp, const uint8_t* Up, const uint8_t* Vp, int ys,
                                                      int cs, int width, int height, uint8_t* out) {
    MP4V_BGR_ROWS_BODY
}
#undef MP4V_BGR_ROWS_BODY

// ------------------------------------------------------------------ decoder
struct Plane {
    int w = 0, h = 0;  // MB-aligned
    std::vector<uint8_t> px;
    uint8_t* row(int y) { return px.data() + (size_t)y * w; }
    const uint8_t* row(int y) const { return px.data() + (size_t)y * w; }
};

struct Frame {
    Plane p[3];
};

struct Decoder {
    // VOL
    int width = 0, height = 0, mb_w = 0, mb_h = 0;
    int time_inc_bits = 1, quant_type = 0, resync_disable = 1, have_vol = 0;
    uint8_t qmat[2][64];  // [intra][raster]
    // VOP
    int qscale = 1, rounding = 0, fcode = 1, dc_thr = 99, vop_type = 0;
    // frames
    Frame cur, ref;
    bool have_ref = false;
    // prediction state (FFmpeg layouts: luma per 8x8 block, b8 stride 2 mb_w + 2 with a
    // one-block border on the left / top / right; chroma per MB, stride mb_w + 2)
    int b8s = 0, cs = 0;
    std::vector<int> dc[3];
    std::vector<int16_t> ac[3];  // 16 per block: [1..7] first column, [9..15] first row
    std::vector<int16_t> mv;     // 2 per luma block
    std::vector<int8_t> mbq;     // qscale per MB (mb_w + 2 stride, border)
    // slice (video packet) state
    int resync_x = 0, resync_y = 0, first_line = 1;
    int mb_x = 0, mb_y = 0;
    // split decode (mvp_mp4v_parse): one MbRec per macroblock and the inverse-quantised
    // coefficients instead of pixels; the device reconstructs (mp4v_recon.hip).  A handle
    // either decodes or parses (mode 1 / 2), never both: parsing leaves the host pictures stale.
    int mode = 0;
    MbRec* rec = nullptr;
    uint32_t* coef = nullptr;
    size_t coef_n = 0, coef_cap = 0;
    int vop_coded = -1;

    MbRec& cur_rec() { return rec[(size_t)mb_y * mb_w + mb_x]; }
    void rec_begin(uint8_t kind) {
        MbRec& r = cur_rec();
        std::memset(&r, 0, sizeof(r));
        r.kind = kind;
        r.coef = (uint32_t)coef_n;
    }
    // dequant(blk, false, n) + emit_block for quant_type 0 over the decoded positions only
    void emit_inter_h263(int n, const int16_t* blk, const uint8_t* pos, int np) {
        const int qmul = qscale << 1, qadd = (qscale - 1) | 1;
        MVP_REQUIRE(coef_n + np <= coef_cap, "mvp_mp4v_parse: coefficient buffer full (%zu entries)", coef_cap);
        int k = 0;
        for (int i = 0; i < np; i++) {
            const int l = blk[pos[i]];
            if (!l) continue;
            const int v = std::max(-2048, std::min(2047, l < 0 ? l * qmul - qadd : l * qmul + qadd));
            coef[coef_n++] = coef_entry(pos[i], v);
            k++;
        }
        cur_rec().nnz[n] = (uint8_t)k;
    }
    // dequant(blk, true, n) + emit_block for quant_type 0 over the positions in mask m (raster order)
    void emit_intra_h263(int n, const int16_t* blk, uint64_t m) {
        const int qmul = qscale << 1, qadd = (qscale - 1) | 1;
        MVP_REQUIRE(coef_n + 64 <= coef_cap, "mvp_mp4v_parse: coefficient buffer full (%zu entries)", coef_cap);
        int k = 0;
        while (m) {
            const int i = __builtin_ctzll(m);
            m &= m - 1;
            const int l = blk[i];
            if (!l) continue;
            const int v = i == 0 ? (int16_t)(l * dc_scale(qscale, n < 4))
                                 : std::max(-2048, std::min(2047, l < 0 ? l * qmul - qadd : l * qmul + qadd));
            if (!v) continue;
            coef[coef_n++] = coef_entry(i, v);
            k++;
        }
        cur_rec().nnz[n] = (uint8_t)k;
    }
    void emit_block(int n, const int16_t* blk) {
        int k = 0;
        for (int i = 0; i < 64; i++) {
            if (!blk[i]) continue;
            MVP_REQUIRE(coef_n < coef_cap, "mvp_mp4v_parse: coefficient buffer full (%zu entries)", coef_cap);
            coef[coef_n++] = coef_entry(i, blk[i]);
            k++;
        }
        cur_rec().nnz[n] = (uint8_t)k;
    }

    int lidx(int bx, int by) const { return (by + 1) * b8s + bx + 1; }
    int cidx(int x, int y) const { return (y + 1) * cs + x + 1; }
    int qidx(int x, int y) const { return (y + 1) * (mb_w + 2) + x + 1; }

    void alloc() {
        mb_w = (width + 15) / 16;
        mb_h = (height + 15) / 16;
        for (Frame* f : {&cur, &ref}) {
            f->p[0].w = mb_w * 16;
            f->p[0].h = mb_h * 16;
            f->p[1].w = f->p[2].w = mb_w * 8;
            f->p[1].h = f->p[2].h = mb_h * 8;
            for (auto& pl : f->p) pl.px.assign((size_t)pl.w * pl.h, 128);
        }
        b8s = 2 * mb_w + 2;
        cs = mb_w + 2;
        dc[0].assign((size_t)b8s * (2 * mb_h + 2), 1024);
        ac[0].assign((size_t)b8s * (2 * mb_h + 2) * 16, 0);
        for (int c = 1; c < 3; c++) {
            dc[c].assign((size_t)cs * (mb_h + 2), 1024);
            ac[c].assign((size_t)cs * (mb_h + 2) * 16, 0);
        }
        mv.assign((size_t)b8s * (2 * mb_h + 2) * 2, 0);
        mbq.assign((size_t)(mb_w + 2) * (mb_h + 2), 0);
    }

    // --- headers
    void parse_vol(Bits& b) {
        b.get1();            // random_accessible_vol
        b.get(8);            // video_object_type_indication
        int verid = 1;
        if (b.get1()) {      // is_object_layer_identifier
            verid = (int)b.get(4);
            b.get(3);        // priority
        }
        if (b.get(4) == 15) b.get(16);  // aspect ratio: extended PAR
        if (b.get1()) {      // vol_control_parameters
            const int chroma = (int)b.get(2);
            MVP_REQUIRE(chroma == 1, "mp4v: chroma_format %d (only 4:2:0)", chroma);
            b.get1();        // low_delay
            if (b.get1()) {  // vbv parameters
                b.get(15); b.get1(); b.get(15); b.get1(); b.get(15); b.get1(); b.get(3); b.get(11); b.get1();
                b.get(15); b.get1();
            }
        }
        const int shape = (int)b.get(2);
        MVP_REQUIRE(shape == 0, "mp4v: video_object_layer_shape %d (only rectangular)", shape);
        b.get1();
        const int res = (int)b.get(16);
        MVP_REQUIRE(res > 0, "mp4v: vop_time_increment_resolution 0");
        int bits = 0;
        for (int v = res - 1; v > 0; v >>= 1) bits++;
        time_inc_bits = std::max(bits, 1);
        b.get1();
        if (b.get1()) b.get(time_inc_bits);  // fixed_vop_rate
        b.get1();
        const int vol_w = (int)b.get(13);
        b.get1();
        const int vol_h = (int)b.get(13);
        b.get1();
        MVP_REQUIRE(vol_w > 0 && vol_h > 0 && vol_w <= 8192 && vol_h <= 8192, "mp4v: frame %dx%d", vol_w, vol_h);
        // the caller sizes its output buffers from the first VOL: a later VOL (repeated before
        // I-VOPs by encoders without a global header) must describe the same frame size
        MVP_REQUIRE(!have_vol || (vol_w == width && vol_h == height),
                    "mp4v: VOL changes the frame size from %dx%d to %dx%d inside one stream", width, height,
                    vol_w, vol_h);
        MVP_REQUIRE(b.get1() == 0, "mp4v: interlaced video is not supported");
        b.get1();  // obmc_disable
        const int sprite = (int)b.get(verid == 1 ? 1 : 2);
        MVP_REQUIRE(sprite == 0, "mp4v: sprites (GMC) are not supported");
        MVP_REQUIRE(b.get1() == 0, "mp4v: not_8_bit video is not supported");
        quant_type = b.get1();
        std::memcpy(qmat[1], kDefaultIntraMatrix, 64);
        std::memcpy(qmat[0], kDefaultInterMatrix, 64);
        if (quant_type) {
            for (int t = 1; t >= 0; t--) {
                if (!b.get1()) continue;  // load_*_quant_mat
                int last = 0;
                int i = 0;
                for (; i < 64; i++) {
                    const int v = (int)b.get(8);
                    if (v == 0) break;
                    last = v;
                    qmat[t][tables().scan_zz[i]] = (uint8_t)v;
                }
                for (; i < 64; i++) qmat[t][tables().scan_zz[i]] = (uint8_t)last;
            }
        }
        if (verid != 1) MVP_REQUIRE(b.get1() == 0, "mp4v: quarter-pel motion is not supported");
        MVP_REQUIRE(b.get1() == 1, "mp4v: complexity estimation headers are not supported");
        resync_disable = b.get1();
        MVP_REQUIRE(b.get1() == 0, "mp4v: data partitioning is not supported");
        if (verid != 1) {
            MVP_REQUIRE(b.get1() == 0, "mp4v: newpred is not supported");
            MVP_REQUIRE(b.get1() == 0, "mp4v: reduced-resolution VOPs are not supported");
        }
        MVP_REQUIRE(b.get1() == 0, "mp4v: scalability is not supported");
        // a repeated VOL only refreshes per-VOL state (time_inc_bits, quant matrices, resync):
        // the reference frames survive it, so a following P-VOP or not-coded VOP still
        // predicts from / repeats the previous picture
        if (!have_vol) {
            width = vol_w;
            height = vol_h;
            alloc();
        }
        have_vol = 1;
    }

    // Scan `data` for start codes; VOL headers configure, VOPs decode.  Returns VOPs decoded.
    int feed(const uint8_t* data, size_t n, int* decoded_vop) {
        int vops = 0;
        size_t i = 0;
        while (i + 3 < n) {
            if (!(data[i] == 0 && data[i + 1] == 0 && data[i + 2] == 1)) {
                i++;
                continue;
            }
            const uint8_t code = data[i + 3];
            size_t j = i + 4;  // payload up to the next start code
            while (j + 2 < n && !(data[j] == 0 && data[j + 1] == 0 && data[j + 2] == 1)) j++;
            if (j + 2 >= n) j = n;
            Bits b;
            b.p = data + i + 4;
            b.n = j - (i + 4);
            if (code >= 0x20 && code <= 0x2f) {
                parse_vol(b);
            } else if (code == 0xb6) {
                MVP_REQUIRE(have_vol, "mp4v: VOP before any VOL header");
                // a VOP's payload may contain byte patterns 00 00 01 only at resync markers'
                // positions, never as start codes: decode to the end of this start code's data
                *decoded_vop = decode_vop(b);
                vops++;
            }
            i = j;
        }
        return vops;
    }

    // --- VOP
    int decode_vop(Bits& b) {
        vop_type = (int)b.get(2);
        MVP_REQUIRE(vop_type <= 1, "mp4v: %s-VOPs are not supported (Simple Profile I / P only)",
                    vop_type == 2 ? "B" : "S");
        while (b.get1()) {}  // modulo_time_base
        b.get1();
        b.get(time_inc_bits);
        b.get1();
        vop_coded = 0;
        if (!b.get1()) return 0;  // vop_coded == 0: the previous frame again
        vop_coded = 1;
        MVP_REQUIRE(vop_type == 0 || have_ref, "mp4v: P-VOP without a reference frame");
        if (vop_type == 1) rounding = b.get1();
        dc_thr = kDcThreshold[b.get(3)];
        qscale = (int)b.get(5);
        MVP_REQUIRE(qscale > 0, "mp4v: vop_quant 0");
        if (vop_type == 1) {
            fcode = (int)b.get(3);
            MVP_REQUIRE(fcode > 0, "mp4v: vop_fcode_forward 0");
        }
        std::swap(cur, ref);  // cur becomes the new frame, ref the previous one
        if (rec)
            for (int i = 0; i < mb_w * mb_h; i++) {
                std::memset(&rec[i], 0, sizeof(MbRec));
                rec[i].kind = MB_LOST;
            }
        resync_x = resync_y = 0;
        first_line = 1;
        for (mb_y = 0; mb_y < mb_h; mb_y++) {
            for (mb_x = 0; mb_x < mb_w; mb_x++) {
                if (!(mb_x == 0 && mb_y == 0) && !resync_disable && at_resync(b)) video_packet_header(b);
                if (resync_x == mb_x && resync_y + 1 == mb_y) first_line = 0;
                MVP_REQUIRE(b.left() > 0, "mp4v: VOP data ends at macroblock (%d, %d)", mb_x, mb_y);
                if (vop_type == 0) decode_mb_intra_vop(b);
                else decode_mb_p(b);
            }
        }
        have_ref = true;
        return 1;
    }

    bool at_resync(const Bits& b) const {
        // next_resync_marker: stuffing '0' + '1's to the byte boundary, then (16 + fcode - 1 for
        // P, 16 for I) zeros and a one
        Bits t = b;
        const int nb = 8 - (int)(t.pos & 7);
        if ((int)t.show(nb) != (1 << (nb - 1)) - 1) return false;
        t.skip(nb);
        const int len = 17 + (vop_type == 1 ? fcode - 1 : 0);
        return t.left() >= len && t.show(std::min(len, 25)) == 1u;
    }

    void video_packet_header(Bits& b) {
        b.align();
        b.skip(17 + (vop_type == 1 ? fcode - 1 : 0));
        int nbits = 0;
        for (int v = mb_w * mb_h - 1; v > 0; v >>= 1) nbits++;
        const int mbn = (int)b.get(std::max(nbits, 1));
        MVP_REQUIRE(mbn < mb_w * mb_h, "mp4v: video packet macroblock_number %d", mbn);
        const int q = (int)b.get(5);
        if (q) qscale = q;
        if (b.get1()) {  // header_extension_code
            while (b.get1()) {}
            b.get1();
            b.get(time_inc_bits);
            b.get1();
            b.get(2);
            dc_thr = kDcThreshold[b.get(3)];
            if (vop_type == 1) b.get(3);
        }
        // macroblocks between the previous position and mbn are lost (corrupt stream): keep going
        mb_x = mbn % mb_w;
        mb_y = mbn / mb_w;
        resync_x = mb_x;
        resync_y = mb_y;
        first_line = 1;
    }

    static int dc_scale(int q, bool luma) {
        if (luma) return q < 5 ? 8 : q < 9 ? 2 * q : q < 25 ? q + 8 : 2 * q - 16;
        return q < 5 ? 8 : q < 25 ? (q + 13) / 2 : q - 6;
    }

    // the six blocks' prediction storage of the current MB
    int* dcp(int n) {
        if (n < 4) return &dc[0][lidx(2 * mb_x + (n & 1), 2 * mb_y + (n >> 1))];
        return &dc[n - 3][cidx(mb_x, mb_y)];
    }
    int16_t* acp(int n) {
        if (n < 4) return &ac[0][(size_t)lidx(2 * mb_x + (n & 1), 2 * mb_y + (n >> 1)) * 16];
        return &ac[n - 3][(size_t)cidx(mb_x, mb_y) * 16];
    }
    int wrap(int n) const { return n < 4 ? b8s : cs; }

    // ff_mpeg4_pred_dc: returns the prediction in the quantised domain and the direction
    int pred_dc(int n, int* dir) {
        const int* v = dcp(n);
        const int w = wrap(n);
        int a = v[-1], bb = v[-1 - w], c = v[-w];
        if (first_line && n != 3) {
            if (n != 2) bb = c = 1024;
            if (n != 1 && mb_x == resync_x) bb = a = 1024;
        }
        if (mb_x == resync_x && mb_y == resync_y + 1 && (n == 0 || n == 4 || n == 5)) bb = 1024;
        int pred;
        if (std::abs(a - bb) < std::abs(bb - c)) {
            pred = c;
            *dir = 1;  // from above
        } else {
            pred = a;
            *dir = 0;  // from the left
        }
        const int s = dc_scale(qscale, n < 4);
        return (pred + (s >> 1)) / s;
    }

    void store_dc(int n, int level_q) {
        int level = level_q * dc_scale(qscale, n < 4);
        if (level & ~2047) level = level < 0 ? 0 : 2047;
        *dcp(n) = level;
    }

    // ff_mpeg4_pred_ac on the quantised block (raster), then store the first row / column
    void pred_ac(int n, int dir, bool ac_pred, int16_t* blk) {
        int16_t* a = acp(n);
        if (ac_pred) {
            if (dir == 0) {
                const int16_t* l = a - 16;
                const int ql = mbq[qidx(mb_x - 1, mb_y)];
                const bool same = mb_x == 0 || qscale == ql || n == 1 || n == 3;
                for (int i = 1; i < 8; i++)
                    blk[i * 8] = (int16_t)(blk[i * 8] + (same ? l[i] : rdiv(l[i] * ql, qscale)));
            } else {
                const int16_t* t = a - 16 * wrap(n);
                const int qt = mbq[qidx(mb_x, mb_y - 1)];
                const bool same = mb_y == 0 || qscale == qt || n == 2 || n == 3;
                for (int i = 1; i < 8; i++) blk[i] = (int16_t)(blk[i] + (same ? t[8 + i] : rdiv(t[8 + i] * qt, qscale)));
            }
        }
        for (int i = 1; i < 8; i++) {
            a[i] = blk[i * 8];
            a[8 + i] = blk[i];
        }
    }
    static int rdiv(int a, int b) { return (a >= 0 ? a + (b >> 1) : a - (b >> 1)) / b; }

    // TCOEF events into blk (raster) through `scan`, starting at scan position `i`; pos (optional):
    // the raster positions written, *npos of them (a position is written at most once)
    void decode_ac(Bits& b, int16_t* blk, bool intra, int i, const uint8_t* scan, uint8_t* pos = nullptr,
                   int* npos = nullptr) {
        const Tables& T = tables();
        const Vlc& vlc = intra ? T.tc_intra : T.tc_inter;
        const int8_t* runs = intra ? kRunIntra : kRunInter;
        const int8_t* levs = intra ? kLevelIntra : kLevelInter;
        const int nl = intra ? kTcoefNotLastIntra : kTcoefNotLastInter;
        const int t = intra ? 1 : 0;
        for (;;) {
            int s = vlc.decode(b);
            MVP_REQUIRE(s >= 0, "mp4v: invalid TCOEF code at macroblock (%d, %d)", mb_x, mb_y);
            int run, level, last;
            if (s == kTcoefEvents) {  // escape
                if (!b.get1()) {       // type 1: level + LMAX
                    s = vlc.decode(b);
                    MVP_REQUIRE(s >= 0 && s < kTcoefEvents, "mp4v: invalid escape-1 code");
                    last = s >= nl;
                    run = runs[s];
                    level = levs[s] + T.lmax[t][last][run];
                    if (b.get1()) level = -level;
                } else if (!b.get1()) {  // type 2: run + RMAX + 1
                    s = vlc.decode(b);
                    MVP_REQUIRE(s >= 0 && s < kTcoefEvents, "mp4v: invalid escape-2 code");
                    last = s >= nl;
                    level = levs[s];
                    run = runs[s] + T.rmax[t][last][level] + 1;
                    if (b.get1()) level = -level;
                } else {  // type 3: fixed length
                    last = b.get1();
                    run = (int)b.get(6);
                    MVP_REQUIRE(b.get1(), "mp4v: escape-3 marker");
                    level = b.get_sbits(12);
                    MVP_REQUIRE(b.get1(), "mp4v: escape-3 marker");
                    MVP_REQUIRE(level != 0, "mp4v: escape-3 level 0");
                }
            } else {
                last = s >= nl;
                run = runs[s];
                level = levs[s];
                if (b.get1()) level = -level;
            }
            i += run;
            MVP_REQUIRE(i < 64, "mp4v: run past the block end at macroblock (%d, %d)", mb_x, mb_y);
            blk[scan[i]] = (int16_t)level;
            if (pos) pos[(*npos)++] = scan[i];
            i++;
            if (last) break;
        }
    }

    void dequant(int16_t* blk, bool intra, int n) {
        if (quant_type == 0) {
            const int qmul = qscale << 1, qadd = (qscale - 1) | 1;
            for (int i = intra ? 1 : 0; i < 64; i++) {
                int l = blk[i];
                if (!l) continue;
                l = l < 0 ? l * qmul - qadd : l * qmul + qadd;
                blk[i] = (int16_t)std::max(-2048, std::min(2047, l));
            }
        } else {
            const uint8_t* m = qmat[intra ? 1 : 0];
            int sum = 0;
            for (int i = intra ? 1 : 0; i < 64; i++) {
                int l = blk[i];
                if (!l) continue;
                const int a = std::abs(l);
                int v = intra ? (a * qscale * m[i]) >> 3 : ((2 * a + 1) * qscale * m[i]) >> 4;
                v = std::min(v, l < 0 ? 2048 : 2047);
                blk[i] = (int16_t)(l < 0 ? -v : v);
                sum += blk[i];
            }
            if (intra) sum += blk[0] * dc_scale(qscale, n < 4);
            if ((sum & 1) == 0) blk[63] ^= 1;  // mismatch control
        }
        if (intra) blk[0] = (int16_t)(blk[0] * dc_scale(qscale, n < 4));
    }

    uint8_t* block_dst(Frame& f, int n, int* stride) {
        if (n < 4) {
            Plane& p = f.p[0];
            *stride = p.w;
            return p.row(16 * mb_y + 8 * (n >> 1)) + 16 * mb_x + 8 * (n & 1);
        }
        Plane& p = f.p[n - 3];
        *stride = p.w;
        return p.row(8 * mb_y) + 8 * mb_x;
    }

    void set_qscale(int q) { qscale = std::max(1, std::min(31, q)); }

    void intra_blocks(Bits& b, int cbp, bool ac_pred, bool use_dc_vlc) {
        const Tables& T = tables();
        if (rec) rec_begin(MB_INTRA);
        for (int n = 0; n < 6; n++) {
            alignas(16) int16_t blk[64] = {};
            int dir = 0;
            const int pred = pred_dc(n, &dir);
            const uint8_t* scan = ac_pred ? (dir == 0 ? T.scan_v : T.scan_h) : T.scan_zz;
            int start = 0;
            if (use_dc_vlc) {
                const int size = (n < 4 ? T.dc_lum : T.dc_chrom).decode(b);
                MVP_REQUIRE(size >= 0, "mp4v: invalid dct_dc_size at macroblock (%d, %d)", mb_x, mb_y);
                int diff = size ? b.get_xbits(size) : 0;
                if (size > 8) MVP_REQUIRE(b.get1(), "mp4v: DC marker bit");
                blk[0] = (int16_t)diff;
                start = 1;
            }
            const bool fast = rec && quant_type == 0;
            uint8_t pos[64];
            int np = 0;
            if (cbp & (32 >> n)) decode_ac(b, blk, true, start, scan, fast ? pos : nullptr, &np);
            const int qdc = blk[0] + pred;
            blk[0] = (int16_t)qdc;
            store_dc(n, qdc);
            pred_ac(n, dir, ac_pred, blk);
            if (fast) {
                // the positions that can be non-zero: the DC, the decoded ones, and the first
                // column (prediction from the left) or row (from above) AC prediction wrote
                uint64_t m = 1;
                for (int i = 0; i < np; i++) m |= 1ull << pos[i];
                if (ac_pred) m |= dir == 0 ? 0x0101010101010100ull : 0xFEull;
                emit_intra_h263(n, blk, m);
                continue;
            }
            dequant(blk, true, n);
            if (rec) {
                emit_block(n, blk);
                continue;
            }
            int stride;
            uint8_t* d = block_dst(cur, n, &stride);
            idct_write(blk, d, stride, false);
        }
    }

    void clear_intra_state() {  // a non-intra MB: DC 1024, AC 0 for its neighbours
        for (int n = 0; n < 6; n++) {
            *dcp(n) = 1024;
            std::memset(acp(n), 0, 16 * sizeof(int16_t));
        }
    }

    void decode_mb_intra_vop(Bits& b) {
        const Tables& T = tables();
        int mcbpc;
        do {
            mcbpc = T.mcbpc_i.decode(b);
            MVP_REQUIRE(mcbpc >= 0, "mp4v: invalid I-VOP MCBPC at macroblock (%d, %d)", mb_x, mb_y);
        } while (mcbpc == 8);  // stuffing
        const bool ac_pred = b.get1();
        const int cbpy = T.cbpy.decode(b);
        MVP_REQUIRE(cbpy >= 0, "mp4v: invalid CBPY");
        const bool use_dc_vlc = qscale < dc_thr;  // the running QP, before this MB's dquant
        if (mcbpc & 4) set_qscale(qscale + dquant(b));
        mbq[qidx(mb_x, mb_y)] = (int8_t)qscale;
        set_mv_all(0, 0);
        intra_blocks(b, (cbpy << 2) | (mcbpc & 3), ac_pred, use_dc_vlc);
    }

    static int dquant(Bits& b) {
        static const int t[4] = {-1, -2, 1, 2};
        return t[b.get(2)];
    }

    int16_t* mvp(int blk) { return &mv[(size_t)lidx(2 * mb_x + (blk & 1), 2 * mb_y + (blk >> 1)) * 2]; }
    void set_mv_all(int x, int y) {
        for (int q = 0; q < 4; q++) {
            int16_t* m = mvp(q);
            m[0] = (int16_t)x;
            m[1] = (int16_t)y;
        }
    }
    static int mid3(int a, int b, int c) { return std::max(std::min(a, b), std::min(std::max(a, b), c)); }

    // ff_h263_pred_motion
    void pred_mv(int block, int* px, int* py) {
        static const int off[4] = {2, 1, 1, -1};
        int16_t* m = mvp(block);
        const int w = b8s * 2;  // int16 pairs
        int16_t* A = m - 2;
        if (first_line && block < 3) {
            if (block == 0) {
                if (mb_x == resync_x) {
                    *px = *py = 0;
                } else if (mb_x + 1 == resync_x) {
                    const int16_t* C = m + 2 * off[block] - w;
                    if (mb_x == 0) {
                        *px = C[0];
                        *py = C[1];
                    } else {
                        *px = mid3(A[0], 0, C[0]);
                        *py = mid3(A[1], 0, C[1]);
                    }
                } else {
                    *px = A[0];
                    *py = A[1];
                }
            } else if (block == 1) {
                if (mb_x + 1 == resync_x) {
                    const int16_t* C = m + 2 * off[block] - w;
                    *px = mid3(A[0], 0, C[0]);
                    *py = mid3(A[1], 0, C[1]);
                } else {
                    *px = A[0];
                    *py = A[1];
                }
            } else {
                const int16_t* B = m - w;
                const int16_t* C = m + 2 * off[block] - w;
                if (mb_x == resync_x) A[0] = A[1] = 0;
                *px = mid3(A[0], B[0], C[0]);
                *py = mid3(A[1], B[1], C[1]);
            }
        } else {
            const int16_t* B = m - w;
            const int16_t* C = m + 2 * off[block] - w;
            *px = mid3(A[0], B[0], C[0]);
            *py = mid3(A[1], B[1], C[1]);
        }
    }

    int decode_mv_component(Bits& b, int pred) {
        const int code = tables().mvd.decode(b);
        MVP_REQUIRE(code >= 0, "mp4v: invalid MVD code at macroblock (%d, %d)", mb_x, mb_y);
        if (code == 0) return pred;
        const int sign = b.get1();
        const int shift = fcode - 1;
        int val = code;
        if (shift) {
            val = (val - 1) << shift;
            val |= (int)b.get(shift);
            val++;
        }
        if (sign) val = -val;
        val += pred;
        const int bits = 5 + fcode;  // sign_extend(val, 5 + f_code)
        val &= (1 << bits) - 1;
        return val >= (1 << (bits - 1)) ? val - (1 << bits) : val;
    }

    // half-pel block prediction from the reference plane with edge clamping: a window of
    // (w + 1) x (h + 1) reference pixels (clamped coordinates only when it leaves the frame)
    void mc(int pl, int x0, int y0, int w, int h, int mvx, int mvy, uint8_t* dst, int stride) {
        const Plane& r = ref.p[pl];
        const int vw = pl == 0 ? width : (width + 1) >> 1, vh = pl == 0 ? height : (height + 1) >> 1;
        const int sx = x0 + (mvx >> 1), sy = y0 + (mvy >> 1);
        const int hx = mvx & 1, hy = mvy & 1;
        uint8_t win[17 * 17];
        const uint8_t* src;
        int ss;
        if (sx >= 0 && sy >= 0 && sx + w < vw && sy + h < vh) {
            src = r.row(sy) + sx;
            ss = r.w;
        } else {
            for (int y = 0; y <= h; y++) {
                const uint8_t* row = r.row(std::min(std::max(sy + y, 0), vh - 1));
                for (int x = 0; x <= w; x++) win[y * 17 + x] = row[std::min(std::max(sx + x, 0), vw - 1)];
            }
            src = win;
            ss = 17;
        }
        const int rnd = rounding;
        if (!hx && !hy) {
            for (int y = 0; y < h; y++) std::memcpy(dst + y * stride, src + y * ss, w);
        } else if (hx && !hy) {
            for (int y = 0; y < h; y++)
                for (int x = 0; x < w; x++) dst[y * stride + x] = (uint8_t)((src[y * ss + x] + src[y * ss + x + 1] + 1 - rnd) >> 1);
        } else if (!hx && hy) {
            for (int y = 0; y < h; y++)
                for (int x = 0; x < w; x++)
                    dst[y * stride + x] = (uint8_t)((src[y * ss + x] + src[(y + 1) * ss + x] + 1 - rnd) >> 1);
        } else {
            for (int y = 0; y < h; y++)
                for (int x = 0; x < w; x++)
                    dst[y * stride + x] = (uint8_t)((src[y * ss + x] + src[y * ss + x + 1] + src[(y + 1) * ss + x] +
                                                     src[(y + 1) * ss + x + 1] + 2 - rnd) >> 2);
        }
    }

    static int round_chroma4(int x) {  // ff_h263_round_chroma on the sum of four vectors
        static const uint8_t tab[16] = {0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2};
        return tab[x & 0xf] + ((x >> 3) & ~1);
    }

    void decode_mb_p(Bits& b) {
        const Tables& T = tables();
        if (b.get1()) {  // not_coded: the reference macroblock, MV 0
            set_mv_all(0, 0);
            clear_intra_state();
            mbq[qidx(mb_x, mb_y)] = (int8_t)qscale;
            if (rec) rec_begin(MB_COPY);
            else copy_mb();
            return;
        }
        int mcbpc;
        do {
            mcbpc = T.mcbpc_p.decode(b);
            MVP_REQUIRE(mcbpc >= 0, "mp4v: invalid P-VOP MCBPC at macroblock (%d, %d)", mb_x, mb_y);
        } while (mcbpc == 20);
        const bool intra = (mcbpc & 4) != 0;
        if (intra) {
            const bool ac_pred = b.get1();
            const int cbpy = T.cbpy.decode(b);
            MVP_REQUIRE(cbpy >= 0, "mp4v: invalid CBPY");
            const bool use_dc_vlc = qscale < dc_thr;
            if (mcbpc & 8) set_qscale(qscale + dquant(b));
            mbq[qidx(mb_x, mb_y)] = (int8_t)qscale;
            set_mv_all(0, 0);
            intra_blocks(b, (cbpy << 2) | (mcbpc & 3), ac_pred, use_dc_vlc);
            return;
        }
        const int cbpy = 15 - T.cbpy.decode(b);
        MVP_REQUIRE(cbpy >= 0 && cbpy <= 15, "mp4v: invalid CBPY");
        if (mcbpc & 8) set_qscale(qscale + dquant(b));
        mbq[qidx(mb_x, mb_y)] = (int8_t)qscale;
        const int cbp = (cbpy << 2) | (mcbpc & 3);
        clear_intra_state();
        int mvx[4], mvy[4];
        if (mcbpc & 16) {  // inter4v
            for (int k = 0; k < 4; k++) {
                int px, py;
                pred_mv(k, &px, &py);
                mvx[k] = decode_mv_component(b, px);
                mvy[k] = decode_mv_component(b, py);
                int16_t* m = mvp(k);
                m[0] = (int16_t)mvx[k];
                m[1] = (int16_t)mvy[k];
            }
        } else {
            int px, py;
            pred_mv(0, &px, &py);
            mvx[0] = decode_mv_component(b, px);
            mvy[0] = decode_mv_component(b, py);
            for (int k = 1; k < 4; k++) {
                mvx[k] = mvx[0];
                mvy[k] = mvy[0];
            }
            set_mv_all(mvx[0], mvy[0]);
        }
        int cmx, cmy;
        if (mcbpc & 16) {
            cmx = round_chroma4(mvx[0] + mvx[1] + mvx[2] + mvx[3]);
            cmy = round_chroma4(mvy[0] + mvy[1] + mvy[2] + mvy[3]);
        } else {
            cmx = (mvx[0] >> 1) | (mvx[0] & 1);
            cmy = (mvy[0] >> 1) | (mvy[0] & 1);
        }
        if (rec) {
            rec_begin(MB_INTER);
            MbRec& r = cur_rec();
            for (int k = 0; k < 4; k++) {
                r.mv[k][0] = (int16_t)mvx[k];
                r.mv[k][1] = (int16_t)mvy[k];
            }
            r.cmv[0] = (int16_t)cmx;
            r.cmv[1] = (int16_t)cmy;
            for (int n = 0; n < 6; n++) {
                if (!(cbp & (32 >> n))) continue;
                alignas(16) int16_t blk[64] = {};
                if (quant_type == 0) {
                    // H.263 inverse quantisation touches only the decoded positions: dequantise
                    // and emit those (in decode order) instead of sweeping all 64 twice
                    uint8_t pos[64];
                    int np = 0;
                    decode_ac(b, blk, false, 0, tables().scan_zz, pos, &np);
                    emit_inter_h263(n, blk, pos, np);
                    continue;
                }
                decode_ac(b, blk, false, 0, tables().scan_zz);
                dequant(blk, false, n);
                emit_block(n, blk);
            }
            return;
        }
        // prediction
        int ls;
        uint8_t* ld = block_dst(cur, 0, &ls);
        if (mcbpc & 16) {
            for (int k = 0; k < 4; k++)
                mc(0, 16 * mb_x + 8 * (k & 1), 16 * mb_y + 8 * (k >> 1), 8, 8, mvx[k], mvy[k],
                   ld + 8 * (k >> 1) * ls + 8 * (k & 1), ls);
        } else {
            mc(0, 16 * mb_x, 16 * mb_y, 16, 16, mvx[0], mvy[0], ld, ls);
        }
        for (int c = 1; c < 3; c++) {
            int s;
            uint8_t* d = block_dst(cur, c + 3, &s);
            mc(c, 8 * mb_x, 8 * mb_y, 8, 8, cmx, cmy, d, s);
        }
        // residual
        for (int n = 0; n < 6; n++) {
            if (!(cbp & (32 >> n))) continue;
            alignas(16) int16_t blk[64] = {};
            decode_ac(b, blk, false, 0, tables().scan_zz);
            dequant(blk, false, n);
            int stride;
            uint8_t* d = block_dst(cur, n, &stride);
            idct_write(blk, d, stride, true);
        }
    }

    void copy_mb() {
        for (int pl = 0; pl < 3; pl++) {
            const int sz = pl == 0 ? 16 : 8;
            Plane& c = cur.p[pl];
            const Plane& r = ref.p[pl];
            for (int y = 0; y < sz; y++)
                std::memcpy(c.row(sz * mb_y + y) + sz * mb_x, r.row(sz * mb_y + y) + sz * mb_x, sz);
        }
    }

    // outputs of the frame last decoded (cur after a coded VOP, or the unchanged frame)
    void write_yuv(uint8_t* out) const {
        const Frame& f = cur;
        uint8_t* o = out;
        for (int pl = 0; pl < 3; pl++) {
            const int w = pl ? (width + 1) >> 1 : width, h = pl ? (height + 1) >> 1 : height;
            for (int y = 0; y < h; y++) {
                std::memcpy(o, f.p[pl].row(y), w);
                o += w;
            }
        }
    }

    void write_bgr(uint8_t* out) const {
        // per-component tables (BT.601 limited range, 8-bit fixed point): y298[Y], then the
        // chroma terms shared by each 2 x 2 luma quad
        const Frame& f = cur;
        const uint8_t *Y = f.p[0].row(0), *U = f.p[1].row(0), *V = f.p[2].row(0);
        if (__builtin_cpu_supports("avx2"))
            bgr_rows_x86avx2(Y, U, V, f.p[0].w, f.p[1].w, width, height, out);
        else
            bgr_rows_plain(Y, U, V, f.p[0].w, f.p[1].w, width, height, out);
    }
};

// Properties a transcription error of the tables would break (see mp4v_tables.h).
int selfcheck() {
    auto prefix_free = [](const Code* c, int n, double* kraft) {
        *kraft = 0;
        for (int i = 0; i < n; i++) {
            if (!c[i].len) continue;
            *kraft += 1.0 / (double)(1u << c[i].len);
            for (int j = 0; j < n; j++) {
                if (i == j || !c[j].len || c[j].len < c[i].len) continue;
                if ((c[j].code >> (c[j].len - c[i].len)) == c[i].code) return false;
            }
        }
        return true;
    };
    struct T {
        const Code* c;
        int n;
        double kmin;
    } ts[] = {{kMcbpcIntra, 9, 0.98}, {kMcbpcInter, 28, 0.998}, {kCbpy, 16, 0.96}, {kMvd, 33, 0.999},
              {kDcLum, 13, 0.999}, {kDcChrom, 13, 0.999}, {kTcoefIntra, kTcoefEvents + 1, 0.998},
              {kTcoefInter, kTcoefEvents + 1, 0.998}};
    int bad = 0;
    for (const T& t : ts) {
        double k;
        if (!prefix_free(t.c, t.n, &k) || k > 1.0 || k < t.kmin) bad |= 1;
    }
    // intra codes = a permutation of the inter codes
    std::vector<uint32_t> a, b;
    for (int i = 0; i <= kTcoefEvents; i++) {
        a.push_back((uint32_t)kTcoefIntra[i].code << 8 | kTcoefIntra[i].len);
        b.push_back((uint32_t)kTcoefInter[i].code << 8 | kTcoefInter[i].len);
    }
    std::sort(a.begin(), a.end());
    std::sort(b.begin(), b.end());
    if (a != b) bad |= 2;
    // (last, run, level) in lexicographic order with levels 1..LMAX contiguous per run
    for (int t = 0; t < 2; t++) {
        const int8_t* run = t ? kRunIntra : kRunInter;
        const int8_t* lev = t ? kLevelIntra : kLevelInter;
        const int nl = t ? kTcoefNotLastIntra : kTcoefNotLastInter;
        for (int i = 0; i < kTcoefEvents; i++) {
            const bool first = i == 0 || i == nl || run[i] != run[i - 1];
            if (first ? lev[i] != 1 : (run[i] != run[i - 1] || lev[i] != lev[i - 1] + 1)) bad |= 4;
            if (!first && i != nl && run[i] < run[i - 1]) bad |= 4;
        }
    }
    // scans are permutations
    for (const uint8_t* s : {kZigzag, kAltHorizontal}) {
        uint64_t seen = 0;
        for (int i = 0; i < 64; i++) seen |= 1ull << s[i];
        if (seen != ~0ull) bad |= 8;
    }
    return bad;
}

}  // namespace mp4v

extern "C" int mvp_mp4v_create(const uint8_t* config, size_t config_bytes, void** handle, int* width, int* height) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(handle && width && height, "mvp_mp4v_create: NULL output pointer");
    auto* d = new mp4v::Decoder;
    try {
        int dummy = 0;
        if (config && config_bytes) d->feed(config, config_bytes, &dummy);
        MVP_REQUIRE(d->have_vol, "mvp_mp4v_create: no video object layer header in the %zu config bytes",
                    config_bytes);
    } catch (...) {
        delete d;
        throw;
    }
    *handle = d;
    *width = d->width;
    *height = d->height;
    MVP_ABI_END
}

extern "C" int mvp_mp4v_decode(void* handle, const uint8_t* data, size_t bytes, uint8_t* bgr_out, uint8_t* yuv_out,
                               int* vops_out) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(handle && data, "mvp_mp4v_decode: NULL pointer");
    auto* d = static_cast<mp4v::Decoder*>(handle);
    MVP_REQUIRE(d->mode != 2, "mvp_mp4v_decode: this handle parses (mvp_mp4v_parse); its pictures are not kept");
    d->mode = 1;
    int coded = 0;
    const int vops = d->feed(data, bytes, &coded);
    MVP_REQUIRE(d->have_ref, "mvp_mp4v_decode: no frame decoded yet");
    if (bgr_out) d->write_bgr(bgr_out);
    if (yuv_out) d->write_yuv(yuv_out);
    if (vops_out) *vops_out = vops;
    MVP_ABI_END
}

extern "C" int mvp_mp4v_parse(void* handle, const uint8_t* data, size_t bytes, void* rec_out, int64_t rec_cap,
                              uint32_t* coef_out, int64_t coef_cap, int64_t* n_coef, int* vop_out) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(handle && data && rec_out && coef_out && n_coef && vop_out, "mvp_mp4v_parse: NULL pointer");
    auto* d = static_cast<mp4v::Decoder*>(handle);
    MVP_REQUIRE(d->mode != 1, "mvp_mp4v_parse: this handle decodes (mvp_mp4v_decode)");
    d->mode = 2;
    MVP_REQUIRE(rec_cap >= (int64_t)d->mb_w * d->mb_h, "mvp_mp4v_parse: %lld records for %d macroblocks",
                (long long)rec_cap, d->mb_w * d->mb_h);
    d->rec = static_cast<mp4v::MbRec*>(rec_out);
    d->coef = coef_out;
    d->coef_n = 0;
    d->coef_cap = (size_t)std::max<int64_t>(coef_cap, 0);
    d->vop_coded = -1;
    int coded = 0;
    int vops = 0;
    try {
        vops = d->feed(data, bytes, &coded);
    } catch (...) {
        d->rec = nullptr;
        d->coef = nullptr;
        throw;
    }
    d->rec = nullptr;
    d->coef = nullptr;
    MVP_REQUIRE(vops <= 1, "mvp_mp4v_parse: %d VOPs in one sample (the split decode takes one per sample)", vops);
    *n_coef = (int64_t)d->coef_n;
    vop_out[0] = vops ? d->vop_coded : -1;
    vop_out[1] = d->rounding;
    MVP_ABI_END
}

extern "C" int mvp_mp4v_parse_many(void* handle, int n, const uint8_t* const* data, const size_t* bytes, void* rec_out,
                                   uint32_t* coef_out, int64_t coef_cap, int64_t* n_coef, int* vop_out, int* n_done) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(handle && n >= 0 && (n == 0 || (data && bytes && rec_out && coef_out && n_coef && vop_out)) && n_done,
                "mvp_mp4v_parse_many: NULL pointer");
    auto* d = static_cast<mp4v::Decoder*>(handle);
    const int64_t n_mb = (int64_t)d->mb_w * d->mb_h, worst = n_mb * 384;
    int64_t used = 0;
    int k = 0;
    *n_done = 0;
    for (; k < n && coef_cap - used >= worst; k++) {
        const int rc = mvp_mp4v_parse(handle, data[k], bytes[k], static_cast<uint8_t*>(rec_out) + k * n_mb * 32, n_mb,
                                      coef_out + used, coef_cap - used, &n_coef[k], &vop_out[2 * k]);
        if (rc != MVP_OK) return rc;  // mvp_last_error() holds the sample's message
        used += n_coef[k];
        *n_done = k + 1;
    }
    MVP_ABI_END
}

extern "C" int mvp_mp4v_destroy(void* handle) {
    MVP_ABI_BEGIN
    delete static_cast<mp4v::Decoder*>(handle);
    MVP_ABI_END
}

extern "C" int mvp_mp4v_selfcheck(void) {
    MVP_ABI_BEGIN
    const int bad = mp4v::selfcheck();
    MVP_REQUIRE(bad == 0, "mvp_mp4v_selfcheck: table check failed (mask %d)", bad);
    MVP_ABI_END
}
