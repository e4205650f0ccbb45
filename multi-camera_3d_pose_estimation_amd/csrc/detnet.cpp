// Person-detector graph runtime (RTMDet-m): validation, liveness-based arena planning,
// launch.  The op list comes from the host builder (mvpose/rtmdet.py); tensors are bf16
// NHWC per image, ops address channel slices ("views") so every concatenation of the
// network (CSP layers, SPP, the PAFPN's top-down / bottom-up joins, the head's cls/reg
// pair) is a shared buffer its producers write into.
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "conv.h"
#include "det.h"
#include "mvp_common.h"

namespace mvp {
namespace {

struct DetNet {
    std::vector<mvp_tensor_desc> tensors;
    std::vector<mvp_det_op> ops;
    int input = 0, size = 0, n_priors = 0, max_batch = 0, max_ca = 8;
    const uint16_t* wb = nullptr;
    const float* fb = nullptr;
    std::vector<int64_t> offset;
    int64_t arena_bytes = 0;
    char* arena = nullptr;
    float* ca_scratch = nullptr;
    std::vector<uint16_t*> wimg;   // per conv op: the GEMM kernel's weight image (owned)
    std::vector<uint16_t*> wband;  // per band-eligible conv op: the band kernel's weight image (owned)
    // producer passes folded into their consumer 1x1 conv (det.h DetConvFold; plan_folds)
    std::vector<int> fold_src;  // per conv op: the DET_UP2 / DET_CA op folded into it, or -1
    std::vector<char> folded;   // per op: its pass runs inside its consumer (UP2: not launched; CA: no scale pass)
    bool lb_folded = false;     // the letterbox runs inside op 0 (the stem stages its rows from the frames)
};

void free_det(DetNet& g) {
    if (g.arena) (void)hipFree(g.arena);
    if (g.ca_scratch) (void)hipFree(g.ca_scratch);
    for (uint16_t* p : g.wimg)
        if (p) (void)hipFree(p);
    for (uint16_t* p : g.wband)
        if (p) (void)hipFree(p);
    g.arena = nullptr;
    g.ca_scratch = nullptr;
    g.wimg.clear();
    g.wband.clear();
}

int64_t per_image_bytes(const mvp_tensor_desc& t) { return (int64_t)t.h * t.w * t.c * 2; }

void validate(DetNet& g, int64_t w_elems, int64_t f_elems) {
    const int nt = (int)g.tensors.size();
    auto view_ok = [&](const mvp_det_view& v, const char* what, size_t k) {
        MVP_REQUIRE(v.t >= 0 && v.t < nt, "det op %zu: %s tensor %d out of range", k, what, v.t);
        const mvp_tensor_desc& t = g.tensors[v.t];
        MVP_REQUIRE(v.coff >= 0 && v.c > 0 && v.coff + v.c <= t.c && v.coff % 8 == 0 && v.c % 8 == 0 && t.c % 8 == 0,
                    "det op %zu: %s view [%d, +%d) of a %d-channel tensor", k, what, v.coff, v.c, t.c);
        return t;
    };
    auto f_ok = [&](int64_t off, int64_t n, size_t k) {
        MVP_REQUIRE(off >= 0 && off % 4 == 0 && off + n <= f_elems, "det op %zu: f32 weights out of the blob", k);
    };
    for (const mvp_tensor_desc& t : g.tensors)
        MVP_REQUIRE(t.h > 0 && t.w > 0 && t.c > 0 && t.c % 4 == 0, "det: bad tensor %dx%dx%d", t.h, t.w, t.c);
    const mvp_tensor_desc& in = g.tensors[g.input];
    MVP_REQUIRE(in.h == g.size && in.w == g.size && in.c == 4, "det: input tensor must be size x size x 4");
    int priors = 0;
    for (size_t k = 0; k < g.ops.size(); k++) {
        const mvp_det_op& op = g.ops[k];
        switch (op.kind) {
            case MVP_DET_STEM: {
                MVP_REQUIRE(op.in.t == g.input && op.in.coff == 0, "det stem %zu: must read the letterboxed input", k);
                const mvp_tensor_desc& o = view_ok(op.out, "out", k);
                MVP_REQUIRE(o.c == 32 && op.out.c == 32 && o.h == g.size / 2 && o.w == g.size / 2,
                            "det stem %zu: output must be a dense size/2 x size/2 x 32 tensor", k);
                f_ok(op.w_off, 32 * 36, k);
                f_ok(op.b_off, 32, k);
                break;
            }
            case MVP_DET_CONV: {
                const mvp_tensor_desc& x = view_ok(op.in, "in", k);
                const mvp_tensor_desc& y = view_ok(op.out, "out", k);
                MVP_REQUIRE(op.ks == 1 || op.ks == 3, "det conv %zu: ks %d", k, op.ks);
                MVP_REQUIRE(op.stride == 1 || (op.stride == 2 && op.ks == 3), "det conv %zu: stride", k);
                MVP_REQUIRE(op.in.c % 32 == 0, "det conv %zu: cin %d not a multiple of 32", k, op.in.c);
                const int pad = op.ks / 2;
                MVP_REQUIRE(y.h == (x.h + 2 * pad - op.ks) / op.stride + 1 && y.w == (x.w + 2 * pad - op.ks) / op.stride + 1,
                            "det conv %zu: output plane", k);
                MVP_REQUIRE(op.in.t != op.out.t, "det conv %zu: a conv cannot write its input tensor", k);
                MVP_REQUIRE(op.aux >= 0 && op.aux <= op.out.c, "det conv %zu: live couts %lld", k, (long long)op.aux);
                if (op.res.t >= 0) {
                    const mvp_tensor_desc& r = view_ok(op.res, "res", k);
                    MVP_REQUIRE(r.h == y.h && r.w == y.w && op.res.c == op.out.c, "det conv %zu: residual shape", k);
                }
                const int64_t cp = det_cout_pad(op.out.c);
                MVP_REQUIRE(op.w_off >= 0 && op.w_off % 8 == 0 && op.w_off + cp * op.ks * op.ks * op.in.c <= w_elems,
                            "det conv %zu: weights out of the bf16 blob", k);
                f_ok(op.b_off, cp, k);
                break;
            }
            case MVP_DET_DW: {
                const mvp_tensor_desc& x = view_ok(op.in, "in", k);
                const mvp_tensor_desc& y = view_ok(op.out, "out", k);
                MVP_REQUIRE(op.ks == 5 && op.stride == 1 && x.h == y.h && x.w == y.w && op.in.c == op.out.c,
                            "det dw %zu: 5x5/s1 with equal shapes only", k);
                MVP_REQUIRE(op.in.t != op.out.t, "det dw %zu: cannot run in place", k);
                f_ok(op.w_off, (int64_t)op.in.c * 25, k);
                f_ok(op.b_off, op.in.c, k);
                break;
            }
            case MVP_DET_DWPW: {
                const mvp_tensor_desc& x = view_ok(op.in, "in", k);
                const mvp_tensor_desc& y = view_ok(op.out, "out", k);
                const int C = op.in.c;
                MVP_REQUIRE(det_dwpw_supported(C) && det_cout_pad(op.out.c) == C && op.ks == 5 && x.h == y.h &&
                                x.w == y.w && op.in.t != op.out.t,
                            "det dwpw %zu: C=%d cout=%d ks %d", k, C, op.out.c, op.ks);
                if (op.res.t >= 0) {
                    const mvp_tensor_desc& r = view_ok(op.res, "res", k);
                    MVP_REQUIRE(r.h == y.h && r.w == y.w && op.res.c == op.out.c, "det dwpw %zu: residual shape", k);
                }
                f_ok(op.w_off, (int64_t)C * 25, k);
                f_ok(op.b_off, 2 * (int64_t)C, k);
                MVP_REQUIRE(op.aux >= 0 && op.aux % 8 == 0 && op.aux + (int64_t)C * C <= w_elems,
                            "det dwpw %zu: pointwise weights out of the bf16 blob", k);
                break;
            }
            case MVP_DET_CA: {
                view_ok(op.in, "in", k);
                MVP_REQUIRE(op.in.c / 8 <= 256, "det ca %zu: %d channels", k, op.in.c);
                f_ok(op.w_off, (int64_t)op.in.c * op.in.c, k);
                f_ok(op.b_off, op.in.c, k);
                g.max_ca = std::max(g.max_ca, op.in.c);
                break;
            }
            case MVP_DET_SPP: {
                const mvp_tensor_desc& x = view_ok(op.in, "in", k);
                MVP_REQUIRE(op.in.coff == 0 && x.c == 4 * op.in.c, "det spp %zu: input must be slice 0 of a 4c buffer", k);
                MVP_REQUIRE(x.h * x.w <= 2048, "det spp %zu: plane too large", k);
                break;
            }
            case MVP_DET_UP2: {
                const mvp_tensor_desc& x = view_ok(op.in, "in", k);
                const mvp_tensor_desc& y = view_ok(op.out, "out", k);
                MVP_REQUIRE(y.h == 2 * x.h && y.w == 2 * x.w && op.in.c == op.out.c, "det up2 %zu: shapes", k);
                break;
            }
            case MVP_DET_HEAD: {
                const mvp_tensor_desc& x = view_ok(op.in, "in", k);
                MVP_REQUIRE(op.in.coff == 0 && op.in.c == x.c && x.c % 16 == 0, "det head %zu: [cls | reg] tensor", k);
                MVP_REQUIRE(op.stride > 0 && x.h * op.stride == g.size && x.w * op.stride == g.size,
                            "det head %zu: stride %d", k, op.stride);
                MVP_REQUIRE(op.aux >= 0 && op.aux + (int64_t)x.h * x.w <= g.n_priors, "det head %zu: prior range", k);
                f_ok(op.w_off, 5 * (int64_t)(x.c / 2), k);
                f_ok(op.b_off, 5, k);
                priors += x.h * x.w;
                break;
            }
            default:
                fail(MVP_ERR_ARG, "det op %zu: unknown kind %d", k, op.kind);
        }
        MVP_REQUIRE(op.act >= 0 && op.act <= 2, "det op %zu: act %d", k, op.act);
    }
    MVP_REQUIRE(priors == g.n_priors, "det: head ops write %d priors, n_priors = %d", priors, g.n_priors);
}

// Greedy first-fit placement of the per-batch tensors by lifetime [first, last touch].
void plan(DetNet& g) {
    const int nt = (int)g.tensors.size(), no = (int)g.ops.size();
    std::vector<int> first(nt, no + 1), last(nt, -2);
    auto touch = [&](int t, int k) {
        if (t < 0) return;
        first[t] = std::min(first[t], k);
        last[t] = std::max(last[t], k);
    };
    touch(g.input, -1);  // the letterbox writes it before op 0
    for (int k = 0; k < no; k++) {
        const mvp_det_op& op = g.ops[k];
        touch(op.in.t, k);
        if (op.kind == MVP_DET_STEM || op.kind == MVP_DET_CONV || op.kind == MVP_DET_DW || op.kind == MVP_DET_UP2 ||
            op.kind == MVP_DET_DWPW)
            touch(op.out.t, k);
        if (op.kind == MVP_DET_CONV || op.kind == MVP_DET_DWPW) touch(op.res.t, k);
        // a fold's consumer reads its producer's input in its own launch (plan_folds runs first)
        if (!g.fold_src.empty() && g.fold_src[k] >= 0) touch(g.ops[g.fold_src[k]].in.t, k);
    }
    std::vector<int> order;
    for (int t = 0; t < nt; t++)
        if (last[t] >= -1) order.push_back(t);
    auto bytes = [&](int t) { return (per_image_bytes(g.tensors[t]) * g.max_batch + 255) / 256 * 256; };
    std::sort(order.begin(), order.end(), [&](int a, int b) { return bytes(a) > bytes(b); });
    struct Placed {
        int64_t off, size;
        int first, last;
    };
    std::vector<Placed> placed;
    g.offset.assign(nt, -1);
    int64_t top = 0;
    for (int t : order) {
        const int64_t sz = bytes(t);
        std::vector<Placed> live;
        for (const Placed& p : placed)
            if (!(p.last < first[t] || last[t] < p.first)) live.push_back(p);
        std::sort(live.begin(), live.end(), [](const Placed& a, const Placed& b) { return a.off < b.off; });
        int64_t off = 0;
        for (const Placed& p : live) {
            if (off + sz <= p.off) break;
            off = std::max(off, p.off + p.size);
        }
        placed.push_back({off, sz, first[t], last[t]});
        g.offset[t] = off;
        top = std::max(top, off + sz);
    }
    g.arena_bytes = top;
}

// Folds (round 6), decided once per graph: a DET_UP2 whose output slice only the next 1x1 conv
// reading that tensor consumes (the neck's top-down joins: the conv's pixel DMA addresses the
// half-resolution source instead), and a DET_CA directly followed by the 1x1 conv on its tensor
// (every CSP layer's final_conv: the scales are applied as the pixels land in LDS).  Each stays
// unfolded unless nothing else reads the bytes the fold leaves unwritten or unscaled.
// MVPOSE_DET_FOLD=0 (read here) keeps every producer pass.
void plan_folds(DetNet& g) {
    const int no = (int)g.ops.size();
    g.fold_src.assign(no, -1);
    g.folded.assign(no, 0);
    g.lb_folded = false;
    {
        const char* e = getenv("MVPOSE_DET_FOLD");
        if (e && e[0] == '0') return;
    }
    // the letterbox into the stem: op 0 is the only reader of the letterboxed input
    g.lb_folded = g.ops[0].kind == MVP_DET_STEM;
    for (int k = 1; k < no; k++) {
        const mvp_det_op& op = g.ops[k];
        if (op.in.t == g.input || ((op.kind == MVP_DET_CONV || op.kind == MVP_DET_DWPW) && op.res.t == g.input))
            g.lb_folded = false;
    }
    auto reads = [&](const mvp_det_op& op, int t) {
        if (op.in.t == t) return true;
        return (op.kind == MVP_DET_CONV || op.kind == MVP_DET_DWPW) && op.res.t == t;
    };
    auto writes = [&](const mvp_det_op& op, int t, int c0, int c1) {
        const bool w = op.kind == MVP_DET_STEM || op.kind == MVP_DET_CONV || op.kind == MVP_DET_DW ||
                       op.kind == MVP_DET_UP2 || op.kind == MVP_DET_DWPW;
        if (w && op.out.t == t && op.out.coff < c1 && c0 < op.out.coff + op.out.c) return true;
        // in-place passes on their input view
        return (op.kind == MVP_DET_CA || op.kind == MVP_DET_SPP) && op.in.t == t;
    };
    for (int k = 0; k < no; k++) {
        const mvp_det_op& u = g.ops[k];
        if (u.kind == MVP_DET_UP2) {
            const int t = u.out.t;
            int j = k + 1;
            while (j < no && !reads(g.ops[j], t)) j++;
            if (j == no) continue;
            const mvp_det_op& c = g.ops[j];
            const mvp_tensor_desc& x = g.tensors[c.in.t];
            if (c.kind != MVP_DET_CONV || c.ks != 1 || c.in.t != t || c.in.coff != 0 || u.out.coff != 0 ||
                u.out.c % 32 != 0 || u.out.c > c.in.c || c.res.t == t || g.tensors[u.in.t].c % 8 != 0 ||
                !det_conv_fold_ok(x.h, x.w, c.in.c, c.out.c, 1, false))
                continue;
            bool ok = true;
            for (int m = 0; m < no && ok; m++) {
                if (m == k || m == j) continue;
                if (reads(g.ops[m], t) && m > k) ok = false;  // another reader of the upsample
                // the source must not change between the upsample and its consumer
                if (m > k && m < j && writes(g.ops[m], u.in.t, u.in.coff, u.in.coff + u.in.c)) ok = false;
                if (m > k && m < j && writes(g.ops[m], t, 0, u.out.c)) ok = false;
            }
            if (!ok) continue;
            g.folded[k] = 1;
            g.fold_src[j] = k;
        } else if (u.kind == MVP_DET_CA && k + 1 < no) {
            const mvp_det_op& c = g.ops[k + 1];
            const mvp_tensor_desc& x = g.tensors[u.in.t];
            if (c.kind != MVP_DET_CONV || c.ks != 1 || c.in.t != u.in.t || c.in.coff != u.in.coff || c.in.c != u.in.c ||
                c.res.t == u.in.t || !det_conv_fold_ok(x.h, x.w, c.in.c, c.out.c, 1, true))
                continue;
            bool ok = true;
            for (int m = k + 2; m < no && ok; m++)
                if (reads(g.ops[m], u.in.t)) ok = false;  // a later reader would see unscaled channels
            if (!ok) continue;
            g.folded[k] = 1;
            g.fold_src[k + 1] = k;
        }
    }
}

}  // namespace
}  // namespace mvp

using mvp::DetNet;

extern "C" int mvp_det_create(const mvp_tensor_desc* tensors, int n_tensors, const mvp_det_op* ops, int n_ops,
                              int input_tensor, int size, int n_priors, const uint16_t* w_dev, int64_t w_elems,
                              const float* f_dev, int64_t f_elems, int max_batch, void** handle_out) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(handle_out != nullptr, "mvp_det_create: handle_out is NULL");
    *handle_out = nullptr;
    MVP_REQUIRE(tensors && n_tensors > 0 && ops && n_ops > 0, "mvp_det_create: empty graph");
    MVP_REQUIRE(input_tensor >= 0 && input_tensor < n_tensors, "mvp_det_create: bad input tensor");
    MVP_REQUIRE(size > 0 && size % 32 == 0, "mvp_det_create: size %d must be a multiple of 32", size);
    MVP_REQUIRE(max_batch > 0 && n_priors > 0, "mvp_det_create: max_batch / n_priors");
    MVP_REQUIRE(w_dev && f_dev, "mvp_det_create: NULL weight blob");
    DetNet* g = new DetNet();
    try {
        g->tensors.assign(tensors, tensors + n_tensors);
        g->ops.assign(ops, ops + n_ops);
        g->input = input_tensor;
        g->size = size;
        g->n_priors = n_priors;
        g->max_batch = max_batch;
        g->wb = w_dev;
        g->fb = f_dev;
        mvp::validate(*g, w_elems, f_elems);
        mvp::plan_folds(*g);
        mvp::plan(*g);
        hipError_t e = hipMalloc(&g->arena, g->arena_bytes);
        if (e != hipSuccess)
            mvp::fail(MVP_ERR_NOMEM, "mvp_det_create: arena of %lld bytes: %s", (long long)g->arena_bytes,
                      hipGetErrorString(e));
        MVP_HIP(hipMalloc(&g->ca_scratch, (size_t)max_batch * 17 * g->max_ca * sizeof(float)));  // launch_det_ca scratch
        // conv weight images for the GEMM kernel (the blobs are not rewritten after create)
        g->wimg.assign(g->ops.size(), nullptr);
        g->wband.assign(g->ops.size(), nullptr);
        for (size_t k = 0; k < g->ops.size(); k++) {
            const mvp_det_op& op = g->ops[k];
            if (op.kind == MVP_DET_DWPW) {  // the pointwise weights' GEMM image
                const int C = op.in.c;
                MVP_HIP(hipMalloc(&g->wimg[k], (size_t)C * C * sizeof(uint16_t)));
                mvp::det_pack_gemm_weights(w_dev + op.aux, g->wimg[k], C, C, nullptr);
                continue;
            }
            if (op.kind != MVP_DET_CONV) continue;
            const int npad = mvp::det_cout_pad(op.out.c), K = op.ks * op.ks * op.in.c;
            MVP_HIP(hipMalloc(&g->wimg[k], (size_t)npad * K * sizeof(uint16_t)));
            mvp::det_pack_gemm_weights(w_dev + op.w_off, g->wimg[k], npad, K, nullptr);
            const mvp_tensor_desc& xt = g->tensors[op.in.t];
            if (mvp::det_band_eligible(xt.h, xt.w, op.in.c, npad, op.ks, op.stride)) {
                MVP_HIP(hipMalloc(&g->wband[k], (size_t)mvp::det_band_rows(npad) * K * sizeof(uint16_t)));
                mvp::det_pack_band_weights(w_dev + op.w_off, g->wband[k], npad, op.in.c, nullptr);
            }
        }
        MVP_HIP(hipDeviceSynchronize());
    } catch (...) {
        mvp::free_det(*g);
        delete g;
        throw;
    }
    *handle_out = g;
    MVP_ABI_END
}

namespace mvp {
namespace {

// Letterbox (when begin == 0) and ops [begin, end) on the arena.
void run_ops(DetNet* g, const uint8_t* frames, int n, int h, int w, int begin, int end, float* cand, void* letterboxed,
             hipStream_t s) {
    auto base = [&](int t) -> char* {
        if (t == g->input && letterboxed) return static_cast<char*>(letterboxed);
        return g->arena + g->offset[t];
    };
    auto vp = [&](const mvp_det_view& v) -> uint16_t* { return reinterpret_cast<uint16_t*>(base(v.t)) + v.coff; };
    auto T = [&](int t) -> const mvp_tensor_desc& { return g->tensors[t]; };
    static const float kMean[3] = {103.53f, 116.28f, 123.675f};
    static const float kStd[3] = {57.375f, 57.12f, 58.395f};
    // the letterbox folded into the stem (plan_folds) unless the caller wants the letterboxed image
    const bool lb_fused = begin == 0 && g->lb_folded && !letterboxed;
    if (begin == 0 && !lb_fused) launch_det_letterbox(frames, n, h, w, g->size, kMean, kStd, base(g->input), s);
    for (int k = begin; k < end; k++) {
        const mvp_det_op& op = g->ops[k];
        switch (op.kind) {
            case MVP_DET_STEM:
                if (lb_fused && k == 0)
                    launch_det_letterbox_stem(frames, h, w, kMean, kStd, g->fb + op.w_off, g->fb + op.b_off, vp(op.out), n,
                                              g->size, op.act, s);
                else
                    launch_det_stem(vp(op.in), g->fb + op.w_off, g->fb + op.b_off, vp(op.out), n, g->size, op.act, s);
                break;
            case MVP_DET_CONV: {
                const mvp_tensor_desc& x = T(op.in.t);
                DetConvFold fold;
                if (g->fold_src[k] >= 0) {
                    const mvp_det_op& u = g->ops[g->fold_src[k]];
                    if (u.kind == MVP_DET_UP2) {
                        fold.up = vp(u.in);
                        fold.up_s = T(u.in.t).c;
                        fold.up_c = u.out.c;
                    } else {
                        fold.ca = det_ca_scales(g->ca_scratch, n, op.in.c);
                    }
                }
                launch_det_conv_gemm(vp(op.in), x.c, g->wb + op.w_off, g->fb + op.b_off,
                                     op.res.t >= 0 ? vp(op.res) : nullptr, op.res.t >= 0 ? T(op.res.t).c : 0,
                                     vp(op.out), T(op.out.t).c, n, x.h, x.w, op.in.c, op.out.c, op.ks, op.stride,
                                     op.act, s, g->wimg[k], g->wband[k], (int)op.aux,
                                     g->fold_src[k] >= 0 ? &fold : nullptr);
                break;
            }
            case MVP_DET_DW: {
                const mvp_tensor_desc& x = T(op.in.t);
                launch_det_dw5(vp(op.in), x.c, vp(op.out), T(op.out.t).c, g->fb + op.w_off, g->fb + op.b_off, n, x.h,
                               x.w, op.in.c, op.act, s);
                break;
            }
            case MVP_DET_DWPW: {
                const mvp_tensor_desc& x = T(op.in.t);
                launch_det_dwpw(vp(op.in), x.c, g->fb + op.w_off, g->fb + op.b_off, g->wimg[k],
                                g->fb + op.b_off + op.in.c, op.res.t >= 0 ? vp(op.res) : nullptr,
                                op.res.t >= 0 ? T(op.res.t).c : 0, vp(op.out), T(op.out.t).c, n, x.h, x.w, op.in.c,
                                op.out.c, op.act, op.act, s);
                break;
            }
            case MVP_DET_CA: {
                const mvp_tensor_desc& x = T(op.in.t);
                launch_det_ca(vp(op.in), x.c, n, x.h * x.w, op.in.c, g->fb + op.w_off, g->fb + op.b_off, g->ca_scratch,
                              s, !g->folded[k]);
                break;
            }
            case MVP_DET_SPP: {
                const mvp_tensor_desc& x = T(op.in.t);
                launch_det_spp(vp(op.in), x.c, n, x.h, x.w, op.in.c, s);
                break;
            }
            case MVP_DET_UP2: {
                if (g->folded[k]) break;  // its consumer reads the source (plan_folds)
                const mvp_tensor_desc& x = T(op.in.t);
                launch_det_up2(vp(op.in), x.c, vp(op.out), T(op.out.t).c, n, x.h, x.w, op.in.c, s);
                break;
            }
            case MVP_DET_HEAD: {
                const mvp_tensor_desc& x = T(op.in.t);
                launch_det_head(vp(op.in), x.c, op.in.c / 2, g->fb + op.w_off, g->fb + op.b_off, cand, n, x.h, x.w,
                                op.stride, g->size, g->n_priors, (int)op.aux, s);
                break;
            }
        }
    }
}

DetNet* checked(void* handle, int n, int h, int w) {
    DetNet* g = static_cast<DetNet*>(handle);
    MVP_REQUIRE(g != nullptr, "mvp_det: NULL handle");
    MVP_REQUIRE(n >= 0 && n <= g->max_batch, "mvp_det: batch %d exceeds max_batch %d", n, g->max_batch);
    MVP_REQUIRE(h > 0 && w > 0, "mvp_det: frame %dx%d", h, w);
    return g;
}

}  // namespace
}  // namespace mvp

extern "C" int mvp_det_forward(void* handle, const uint8_t* frames, int n, int h, int w, float score_thr, float* cand,
                               float* best, void* letterboxed, void* stream) {
    MVP_ABI_BEGIN
    DetNet* g = mvp::checked(handle, n, h, w);
    if (n == 0) return MVP_OK;
    MVP_REQUIRE(frames && cand && best, "mvp_det_forward: NULL buffer");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    mvp::run_ops(g, frames, n, h, w, 0, (int)g->ops.size(), cand, letterboxed, s);
    int nh, nw;
    mvp::det_rescale_size(h, w, g->size, nh, nw);
    // mmdet _bbox_post_process: boxes * (1 / scale_factor) with scale_factor = (new_w / w, new_h / h)
    const float fx = (float)(1.0 / ((double)nw / w)), fy = (float)(1.0 / ((double)nh / h));
    mvp::launch_det_select(cand, n, g->n_priors, score_thr, fx, fy, best, s);
    MVP_ABI_END
}

extern "C" int mvp_det_run_ops(void* handle, const uint8_t* frames, int n, int h, int w, int op_begin, int op_end,
                               float* cand, void* stream) {
    MVP_ABI_BEGIN
    DetNet* g = mvp::checked(handle, n, h, w);
    MVP_REQUIRE(op_begin >= 0 && op_begin <= op_end && op_end <= (int)g->ops.size(), "mvp_det_run_ops: op range");
    if (n == 0 || op_begin == op_end) return MVP_OK;
    MVP_REQUIRE((op_begin > 0 || frames) && cand, "mvp_det_run_ops: NULL buffer");
    mvp::run_ops(g, frames, n, h, w, op_begin, op_end, cand, nullptr, reinterpret_cast<hipStream_t>(stream));
    MVP_ABI_END
}

extern "C" int mvp_det_folded_ops(void* handle, int* folded_out, int n_ops) {
    MVP_ABI_BEGIN
    DetNet* g = static_cast<DetNet*>(handle);
    MVP_REQUIRE(g != nullptr && folded_out != nullptr, "mvp_det_folded_ops: NULL argument");
    MVP_REQUIRE(n_ops == (int)g->ops.size(), "mvp_det_folded_ops: %d ops, the graph has %zu", n_ops, g->ops.size());
    for (int k = 0; k < n_ops; k++) folded_out[k] = g->folded[k];
    if (g->lb_folded && n_ops > 0) folded_out[0] = 2;
    MVP_ABI_END
}

extern "C" int mvp_det_tensor_copy(void* handle, int t, int n, void* buf, int to_arena, void* stream) {
    MVP_ABI_BEGIN
    DetNet* g = static_cast<DetNet*>(handle);
    MVP_REQUIRE(g != nullptr, "mvp_det_tensor_copy: NULL handle");
    MVP_REQUIRE(t >= 0 && t < (int)g->tensors.size() && g->offset[t] >= 0, "mvp_det_tensor_copy: tensor %d", t);
    MVP_REQUIRE(n >= 0 && n <= g->max_batch && (n == 0 || buf), "mvp_det_tensor_copy: batch / buffer");
    const size_t bytes = (size_t)n * mvp::per_image_bytes(g->tensors[t]);
    char* a = g->arena + g->offset[t];
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (bytes) MVP_HIP(hipMemcpyAsync(to_arena ? a : buf, to_arena ? buf : a, bytes, hipMemcpyDeviceToDevice, s));
    MVP_ABI_END
}

extern "C" int mvp_det_arena_bytes(void* handle, int64_t* bytes_out) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(handle && bytes_out, "mvp_det_arena_bytes: NULL argument");
    *bytes_out = static_cast<DetNet*>(handle)->arena_bytes;
    MVP_ABI_END
}

extern "C" int mvp_det_destroy(void* handle) {
    MVP_ABI_BEGIN
    DetNet* g = static_cast<DetNet*>(handle);
    if (g) {
        mvp::free_det(*g);
        delete g;
    }
    MVP_ABI_END
}
