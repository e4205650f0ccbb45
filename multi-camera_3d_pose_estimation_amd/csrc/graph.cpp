// Backbone graph runtime: validation, liveness-based arena planning, launch.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "conv.h"
#include "mvp_common.h"

namespace mvp {
namespace {

struct Segment {
    int first_op = 0, last_op = -1;  // inclusive op range
    int micro_batch = 0;             // 0 = whole batch
};

struct Graph {
    std::vector<mvp_tensor_desc> tensors;
    std::vector<mvp_op_desc> ops;
    std::vector<Segment> segs;
    std::vector<int> local_seg;  // segment a tensor is local to (micro-batch sized), -1 = full batch
    int input = -1, output = -1;
    const uint16_t* wb = nullptr;
    const float* fb = nullptr;
    int max_batch = 0;
    std::vector<int> absorbed;    // op folded into another op (fused BasicBlock / cat-fusion), not run on its own
    std::vector<int> block_head;  // op runs the fused BasicBlock of (op - 1, op)
    std::vector<int> cat_src;     // 1x1 op that also computes the absorbed 1x1 op cat_src[k] (-1: none)
    std::vector<uint16_t*> cat_w; // its concatenated weights [cout_pad][cin_k + cin_src] (owned)
    std::vector<float*> cat_b;    // and summed biases [cout_pad] (owned)
    std::vector<int> pair_tail;   // 1x1 op whose 256->64 successor (absorbed) runs in the same launch (-1: none)
    std::vector<int> stem_head;   // 3x3/s2 conv that also runs the (absorbed) stem op stem_head[k] (-1: none)
    std::vector<int> twin;        // 3x3/s1 conv whose (absorbed) 3x3/s2 sibling on the same input runs in its launch
    std::vector<std::vector<int>> sib;  // 3x3/s2 conv whose (absorbed) 3x3/s2 siblings on its input run in its launch
    std::vector<uint16_t*> sib_w;       // their cout-concatenated weights [128][3][3][cin] (owned)
    std::vector<float*> sib_b;          // and biases [128] (owned)
    std::vector<uint16_t*> t16_w;       // tconv16 weight image of a 128/256-ch branch-plane conv (owned)
    std::vector<uint16_t*> tr_w;        // trans1 weight image of a twin-fused transition (owned)
    std::vector<int> head_src;          // heatmap head that also runs the (absorbed) fuse op head_src[k] (-1: none)
    std::vector<int> bneck;             // Bottleneck conv3 whose (absorbed) conv1 bneck[k] and conv2 run in its launch (-1: none)
    std::vector<int> bneck_mid;         // and its (absorbed) conv2
    std::vector<int> bneck_perm;        // its conv1 sums K in the Bottleneck join's order (bneck.hip)
    std::vector<int> bneck_lead;        // layer1's first block: 64-ch input, conv3 cat-fused with the downsample
    std::vector<int> planar;            // bneck head / trans1 twin: its output / input in chunk-planar layout
    std::vector<int64_t> offset;  // per-crop-batch arena offsets (bytes), -1 = external
    int64_t arena_bytes = 0;
    char* arena = nullptr;
};

int64_t elem_size(int dtype) { return dtype == MVP_DT_F32_NCHW ? 4 : 2; }

int64_t tensor_bytes(const mvp_tensor_desc& t, int batch) {
    return (int64_t)batch * t.h * t.w * t.c * elem_size(t.dtype);
}

void validate(Graph& g, int64_t w_elems, int64_t f_elems) {
    const int nt = (int)g.tensors.size();
    auto T = [&](int id) -> const mvp_tensor_desc& {
        MVP_REQUIRE(id >= 0 && id < nt, "graph: tensor id %d out of range", id);
        return g.tensors[id];
    };
    std::vector<int> defined(nt, 0);
    defined[g.input] = 1;
    for (size_t k = 0; k < g.ops.size(); k++) {
        const mvp_op_desc& op = g.ops[k];
        const mvp_tensor_desc& o = T(op.out);
        MVP_REQUIRE(op.n_in >= 1 && op.n_in <= 4, "graph op %zu: n_in=%d", k, op.n_in);
        for (int i = 0; i < op.n_in; i++) {
            if (op.kind == MVP_OP_CONV && i == 1 && op.in[1] < 0) continue;
            T(op.in[i]);
            MVP_REQUIRE(defined[op.in[i]], "graph op %zu reads tensor %d before it is produced", k, op.in[i]);
        }
        MVP_REQUIRE(!defined[op.out], "graph op %zu: tensor %d produced twice", k, op.out);
        if (op.kind == MVP_OP_STEM) {
            const mvp_tensor_desc& x = T(op.in[0]);
            MVP_REQUIRE(x.c == 4 && x.dtype == MVP_DT_BF16_NHWC, "stem: input must be bf16 NHWC with 4 channels");
            MVP_REQUIRE(o.c == 64 && o.h == (x.h - 1) / 2 + 1 && o.w == (x.w - 1) / 2 + 1, "stem: output shape");
            MVP_REQUIRE(op.w_off >= 0 && op.w_off + 64 * 36 <= f_elems && op.b_off >= 0 && op.b_off + 64 <= f_elems,
                        "stem: weights out of the f32 blob");
        } else if (op.kind == MVP_OP_CONV) {
            const mvp_tensor_desc& x = T(op.in[0]);
            const int pad = op.ks / 2;
            MVP_REQUIRE(op.ks == 1 || op.ks == 3, "conv op %zu: ks", k);
            MVP_REQUIRE(op.stride == 1 || (op.stride == 2 && op.ks == 3), "conv op %zu: stride", k);
            MVP_REQUIRE(x.c == op.cin && x.dtype == MVP_DT_BF16_NHWC && op.cin % 32 == 0,
                        "conv op %zu: input channels %d vs cin %d", k, x.c, op.cin);
            MVP_REQUIRE(o.c == op.cout && o.h == (x.h + 2 * pad - op.ks) / op.stride + 1 &&
                            o.w == (x.w + 2 * pad - op.ks) / op.stride + 1,
                        "conv op %zu: output shape", k);
            MVP_REQUIRE(o.dtype == MVP_DT_F32_NCHW || op.cout % 4 == 0, "conv op %zu: cout %% 4", k);
            if (op.n_in > 1 && op.in[1] >= 0) {
                const mvp_tensor_desc& r = T(op.in[1]);
                MVP_REQUIRE(r.h == o.h && r.w == o.w && r.c == o.c && r.dtype == MVP_DT_BF16_NHWC &&
                                o.dtype == MVP_DT_BF16_NHWC,
                            "conv op %zu: residual shape", k);
            }
            const int64_t cp = conv_cout_pad(op.cout);
            MVP_REQUIRE(op.w_off >= 0 && op.w_off % 8 == 0 && op.w_off + cp * op.ks * op.ks * op.cin <= w_elems,
                        "conv op %zu: weights out of the bf16 blob", k);
            MVP_REQUIRE(op.b_off >= 0 && op.b_off % 4 == 0 && op.b_off + cp <= f_elems,
                        "conv op %zu: bias out of the f32 blob", k);
        } else if (op.kind == MVP_OP_FUSE) {
            MVP_REQUIRE(o.dtype == MVP_DT_BF16_NHWC && o.c % 8 == 0, "fuse op %zu: output", k);
            for (int i = 0; i < op.n_in; i++) {
                const mvp_tensor_desc& x = T(op.in[i]);
                const int u = op.up[i];
                MVP_REQUIRE(u >= 1 && x.c == o.c && x.h * u == o.h && x.w * u == o.w, "fuse op %zu: input %d shape",
                            k, i);
            }
        } else {
            fail(MVP_ERR_ARG, "graph op %zu: unknown kind %d", k, op.kind);
        }
        defined[op.out] = 1;
    }
    MVP_REQUIRE(defined[g.output], "graph: output tensor never produced");
    // segments: contiguous op ranges in increasing order
    const int ns = (int)g.segs.size();
    int prev = -1;
    for (int k = 0; k < (int)g.ops.size(); k++) {
        const int sg = g.ops[k].segment;
        MVP_REQUIRE(sg >= 0 && sg < ns, "graph op %d: segment %d out of range", k, sg);
        MVP_REQUIRE(sg >= prev, "graph op %d: segments must be contiguous and ordered", k);
        if (sg != prev) g.segs[sg].first_op = k;
        g.segs[sg].last_op = k;
        prev = sg;
    }
}

// Fusion pass: a 3x3 conv pair conv1 (relu) -> conv2 (+ conv1's input as residual,
// relu) on 32 channels (64x48 plane) or 64 channels (32x24 plane, tblock64.hip) whose
// intermediate feeds nothing else becomes one fused BasicBlock launch; the intermediate
// tensor is then never allocated.
void fuse(Graph& g, bool enable) {
    const int no = (int)g.ops.size(), nt = (int)g.tensors.size();
    g.absorbed.assign(no, 0);
    g.block_head.assign(no, 0);
    if (!enable) return;
    std::vector<int> uses(nt, 0);
    for (const mvp_op_desc& op : g.ops)
        for (int i = 0; i < op.n_in; i++)
            if (op.in[i] >= 0) uses[op.in[i]]++;
    auto is_block_conv3 = [&](const mvp_op_desc& op) {
        return op.kind == MVP_OP_CONV && op.ks == 3 && op.stride == 1 && (op.cin == 32 || op.cin == 64) &&
               op.cout == op.cin && op.relu && g.tensors[op.out].dtype == MVP_DT_BF16_NHWC;
    };
    for (int k = 0; k + 1 < no; k++) {
        const mvp_op_desc& a = g.ops[k];
        const mvp_op_desc& b = g.ops[k + 1];
        if (g.absorbed[k] || g.block_head[k] || !is_block_conv3(a) || !is_block_conv3(b) || a.cin != b.cin) continue;
        const bool a_plain = a.n_in == 1 || a.in[1] < 0;
        const bool b_res = b.n_in > 1 && b.in[1] == a.in[0];
        const mvp_tensor_desc& t = g.tensors[a.out];
        if (!a_plain || !b_res || b.in[0] != a.out || uses[a.out] != 1 || a.out == g.output) continue;
        const bool ok = a.cin == 32 ? basic_block_c32_supported(t.h, t.w) : tblock64_supported(t.h, t.w);
        if (a.segment != b.segment || !ok) continue;
        g.absorbed[k] = 1;
        g.block_head[k + 1] = 1;
        k++;
    }
}

// Cat-fusion pass: y = act(conv1x1_B(h) + bias_B + t) whose residual t = conv1x1_A(x) + bias_A
// (no activation, consumed only here: the Bottleneck downsample) becomes ONE 1x1 conv over
// the channel concatenation [h, x] with weights [W_B | W_A] and bias bias_B + bias_A.  The
// t tensor (256 channels at 64x48 in HRNet-W32: 1.6 GB per 1024 crops, written then read
// back as the residual) disappears, and t is no longer rounded to bf16 before the add.
void cat_fuse(Graph& g, bool enable) {
    const int no = (int)g.ops.size(), nt = (int)g.tensors.size();
    g.cat_src.assign(no, -1);
    g.cat_w.assign(no, nullptr);
    g.cat_b.assign(no, nullptr);
    if (!enable) return;
    std::vector<int> uses(nt, 0), producer(nt, -1);
    for (int k = 0; k < no; k++) {
        const mvp_op_desc& op = g.ops[k];
        producer[op.out] = k;
        for (int i = 0; i < op.n_in; i++)
            if (op.in[i] >= 0 && !(g.block_head[k] && i == 0)) uses[op.in[i]]++;
    }
    auto plain_1x1 = [&](const mvp_op_desc& op) {
        return op.kind == MVP_OP_CONV && op.ks == 1 && op.stride == 1 && op.cin % 32 == 0 &&
               g.tensors[op.out].dtype == MVP_DT_BF16_NHWC;
    };
    for (int b = 0; b < no; b++) {
        const mvp_op_desc& B = g.ops[b];
        if (g.absorbed[b] || g.block_head[b] || !plain_1x1(B) || B.n_in < 2 || B.in[1] < 0) continue;
        const int t = B.in[1], a = producer[t];
        if (a < 0 || a >= b || g.absorbed[a] || g.block_head[a] || g.cat_src[a] >= 0) continue;
        const mvp_op_desc& A = g.ops[a];
        if (!plain_1x1(A) || (A.n_in > 1 && A.in[1] >= 0) || A.relu || A.cout != B.cout) continue;
        if (uses[t] != 1 || t == g.output || A.segment != B.segment) continue;
        const int kch = (A.cin + B.cin) / 32;  // conv1x1_kernel instantiations: K = 32, 64, 128, 256
        if (kch != 2 && kch != 4 && kch != 8) continue;
        g.absorbed[a] = 1;
        g.cat_src[b] = a;
    }
}

// Pair-fusion pass (Bottleneck join): a 1x1 conv A producing 256 channels with ReLU (the
// Bottleneck's conv3, single input + residual or cat-fused with the downsample) whose
// output T is read by a 1x1 conv B (256 -> 64, ReLU, no residual: the next Bottleneck's
// conv1) runs as one conv1x1_pair launch that writes T (still needed as the next
// residual) and B's output; T is no longer re-read for B.
void pair_fuse(Graph& g, bool enable) {
    const int no = (int)g.ops.size(), nt = (int)g.tensors.size();
    g.pair_tail.assign(no, -1);
    if (!enable) return;
    std::vector<int> producer(nt, -1);
    for (int k = 0; k < no; k++) producer[g.ops[k].out] = k;
    auto plain_1x1 = [&](int k) {
        const mvp_op_desc& op = g.ops[k];
        return !g.absorbed[k] && !g.block_head[k] && g.bneck[k] < 0 && op.kind == MVP_OP_CONV && op.ks == 1 &&
               op.stride == 1 &&
               op.relu && g.tensors[op.out].dtype == MVP_DT_BF16_NHWC;
    };
    for (int b = 0; b < no; b++) {
        const mvp_op_desc& B = g.ops[b];
        if (!plain_1x1(b) || (B.n_in > 1 && B.in[1] >= 0) || B.cin != 256 || B.cout != 64) continue;
        const int a = producer[B.in[0]];
        if (a < 0 || a >= b || !plain_1x1(a) || g.pair_tail[a] >= 0) continue;
        const mvp_op_desc& A = g.ops[a];
        const int cin = A.cin + (g.cat_src[a] >= 0 ? g.ops[g.cat_src[a]].cin : 0);
        if (A.cout != 256 || A.segment != B.segment) continue;
        if (!conv1x1_pair_supported(cin, A.cout, B.cout)) continue;
        g.pair_tail[a] = b;
        g.absorbed[b] = 1;
    }
}

// Bottleneck-fusion pass (bneck.hip): layer1's Bottleneck on the 256-ch 64x48 plane — conv1
// (1x1 256 -> 64, ReLU), conv2 (3x3 64 -> 64, ReLU), conv3 (1x1 64 -> 256, + the block's
// input, ReLU), intermediates read by nothing else — runs as one streaming launch; the two
// 64-ch intermediates are never allocated.  Runs before pair_fuse (which would otherwise join
// conv1 to the previous block's conv3); conv1 keeps the K order the join would have given it
// (bneck_perm) so the result stays bit-identical to the unfused graph.
void bneck_fuse(Graph& g, bool enable, bool pair_enabled) {
    const int no = (int)g.ops.size(), nt = (int)g.tensors.size();
    g.bneck.assign(no, -1);
    g.bneck_mid.assign(no, -1);
    g.bneck_perm.assign(no, 0);
    g.bneck_lead.assign(no, 0);
    if (!enable) return;
    std::vector<int> uses(nt, 0), producer(nt, -1);
    for (int k = 0; k < no; k++) {
        const mvp_op_desc& op = g.ops[k];
        producer[op.out] = k;
        for (int i = 0; i < op.n_in; i++)
            if (op.in[i] >= 0 && !(g.block_head[k] && i == 0)) uses[op.in[i]]++;
    }
    auto conv = [&](int k, int ks, int cin, int cout) {
        if (k < 0 || g.absorbed[k] || g.block_head[k] || g.cat_src[k] >= 0) return false;
        const mvp_op_desc& op = g.ops[k];
        return op.kind == MVP_OP_CONV && op.ks == ks && op.stride == 1 && op.relu && op.cin == cin &&
               op.cout == cout && g.tensors[op.out].dtype == MVP_DT_BF16_NHWC;
    };
    auto no_res = [&](int k) { return g.ops[k].n_in < 2 || g.ops[k].in[1] < 0; };
    for (int c = 0; c < no; c++) {
        if (!conv(c, 1, 64, 256) || no_res(c)) continue;
        const mvp_op_desc& C = g.ops[c];
        const int b = producer[C.in[0]];
        if (!conv(b, 3, 64, 64) || !no_res(b) || uses[g.ops[b].out] != 1) continue;
        const int a = producer[g.ops[b].in[0]];
        if (!conv(a, 1, 256, 64) || !no_res(a) || uses[g.ops[a].out] != 1) continue;
        const mvp_op_desc& A = g.ops[a];
        if (A.in[0] != C.in[1] || A.segment != C.segment || g.ops[b].segment != C.segment) continue;
        if (g.ops[b].out == g.output || A.out == g.output) continue;
        const mvp_tensor_desc& x = g.tensors[A.in[0]];
        if (!bneck_supported(x.h, x.w, x.c, A.cout)) continue;
        // would pair_fuse have joined conv1 to its producer (a 1x1 256-cout ReLU conv)?
        int perm = 0;
        const int f = producer[A.in[0]];
        if (pair_enabled && f >= 0 && !g.absorbed[f] && !g.block_head[f]) {
            const mvp_op_desc& F = g.ops[f];
            const int cin = F.cin + (g.cat_src[f] >= 0 ? g.ops[g.cat_src[f]].cin : 0);
            perm = F.kind == MVP_OP_CONV && F.ks == 1 && F.stride == 1 && F.relu && F.cout == 256 &&
                   F.segment == A.segment && g.tensors[F.out].dtype == MVP_DT_BF16_NHWC &&
                   conv1x1_pair_supported(cin, 256, 64);
        }
        g.absorbed[a] = 1;
        g.absorbed[b] = 1;
        g.bneck[c] = a;
        g.bneck_mid[c] = b;
        g.bneck_perm[c] = perm;
    }
    // layer1's first block: conv1 (1x1 64 -> 64) and the downsample (1x1 64 -> 256, cat-fused
    // into conv3) read the same 64-ch tensor; conv3's K is [conv2's output | that tensor]
    for (int c = 0; c < no; c++) {
        const int d = g.cat_src[c];
        if (d < 0 || g.absorbed[c] || g.block_head[c] || g.bneck[c] >= 0) continue;
        const mvp_op_desc& C = g.ops[c];
        if (C.kind != MVP_OP_CONV || C.ks != 1 || C.stride != 1 || !C.relu || C.cin != 64 || C.cout != 256 ||
            g.tensors[C.out].dtype != MVP_DT_BF16_NHWC || g.ops[d].cin != 64)
            continue;
        const int b = producer[C.in[0]];
        if (b < 0 || g.absorbed[b] || g.block_head[b] || g.cat_src[b] >= 0) continue;
        const mvp_op_desc& B = g.ops[b];
        if (B.kind != MVP_OP_CONV || B.ks != 3 || B.stride != 1 || !B.relu || B.cin != 64 || B.cout != 64 ||
            !no_res(b) || uses[B.out] != 1 || B.out == g.output)
            continue;
        const int a = producer[B.in[0]];
        if (a < 0 || g.absorbed[a] || g.block_head[a] || g.cat_src[a] >= 0) continue;
        const mvp_op_desc& A = g.ops[a];
        if (A.kind != MVP_OP_CONV || A.ks != 1 || A.stride != 1 || !A.relu || A.cin != 64 || A.cout != 64 ||
            !no_res(a) || uses[A.out] != 1 || A.out == g.output || A.in[0] != g.ops[d].in[0])
            continue;
        if (A.segment != C.segment || B.segment != C.segment) continue;
        const mvp_tensor_desc& x = g.tensors[A.in[0]];
        if (!bneck_supported(x.h, x.w, x.c, A.cout)) continue;
        g.absorbed[a] = 1;
        g.absorbed[b] = 1;
        g.bneck[c] = a;
        g.bneck_mid[c] = b;
        g.bneck_lead[c] = 1;
    }
}

// Stem-fusion pass: the stem conv (OP_STEM, 4 -> 64, s2) whose output feeds only a
// 3x3/s2 64 -> 64 conv (HRNet's conv2) runs inside that conv's launch (stem2.hip); the
// 128x96x64 intermediate (1.6 GB per 1024 crops) is never allocated.
void stem_fuse(Graph& g, bool enable) {
    const int no = (int)g.ops.size(), nt = (int)g.tensors.size();
    g.stem_head.assign(no, -1);
    if (!enable) return;
    std::vector<int> uses(nt, 0);
    for (const mvp_op_desc& op : g.ops)
        for (int i = 0; i < op.n_in; i++)
            if (op.in[i] >= 0) uses[op.in[i]]++;
    for (int a = 0; a < no; a++) {
        const mvp_op_desc& A = g.ops[a];
        if (A.kind != MVP_OP_STEM || g.absorbed[a] || uses[A.out] != 1 || A.out == g.output) continue;
        for (int b = a + 1; b < no; b++) {
            const mvp_op_desc& B = g.ops[b];
            if (B.in[0] != A.out) continue;
            const mvp_tensor_desc& x = g.tensors[A.in[0]];
            if (B.kind == MVP_OP_CONV && !g.absorbed[b] && !g.block_head[b] && g.cat_src[b] < 0 &&
                g.pair_tail[b] < 0 && B.ks == 3 && B.stride == 2 && B.relu && (B.n_in < 2 || B.in[1] < 0) &&
                B.segment == A.segment && g.tensors[B.out].dtype == MVP_DT_BF16_NHWC &&
                stem2_supported(x.h, x.w, B.cin, B.cout)) {
                g.absorbed[a] = 1;
                g.stem_head[b] = a;
            }
            break;
        }
    }
}

// Transition-fusion pass: HRNet's transition1 reads the layer1 output (256 ch @ 64x48) with
// two 3x3 convs (s1 -> 32 ch, s2 -> 64 ch); trans1.hip runs both from one pass over it.
void twin_fuse(Graph& g, bool enable) {
    const int no = (int)g.ops.size();
    g.twin.assign(no, -1);
    if (!enable) return;
    auto plain3 = [&](int k, int stride) {
        const mvp_op_desc& op = g.ops[k];
        return op.kind == MVP_OP_CONV && !g.absorbed[k] && !g.block_head[k] && g.cat_src[k] < 0 &&
               g.pair_tail[k] < 0 && g.stem_head[k] < 0 && op.ks == 3 && op.stride == stride && op.relu &&
               (op.n_in < 2 || op.in[1] < 0) && g.tensors[op.out].dtype == MVP_DT_BF16_NHWC;
    };
    for (int a = 0; a < no; a++) {
        if (!plain3(a, 1)) continue;
        const mvp_op_desc& A = g.ops[a];
        const mvp_tensor_desc& x = g.tensors[A.in[0]];
        for (int b = a + 1; b < no; b++) {
            const mvp_op_desc& B = g.ops[b];
            if (B.in[0] != A.in[0] || !plain3(b, 2) || B.segment != A.segment) continue;
            if (!trans1_supported(x.h, x.w, x.c, A.cout, B.cout)) continue;
            g.twin[a] = b;
            g.absorbed[b] = 1;
            break;
        }
    }
}

// Planar-layout pass: a fused Bottleneck whose output feeds only a fused transition1 (twin)
// writes it chunk-planar ([N][16][H][W][16]) and trans1 reads it so: each 16-channel item of
// trans1 is then contiguous in HBM instead of a quarter of every 128-B line (PMC: trans1 read
// its 1.6 GB input 1.67 times).  Numerically a no-op.
void planar_fuse(Graph& g) {
    const int no = (int)g.ops.size();
    g.planar.assign(no, 0);
    for (int k = 0; k < no; k++) {
        if (g.bneck[k] < 0 || g.bneck_lead[k]) continue;
        const int t = g.ops[k].out;
        if (t == g.output) continue;
        int tw = -1, ok = 1;
        for (int c = 0; c < no && ok; c++) {
            const mvp_op_desc& op = g.ops[c];
            for (int i = 0; i < op.n_in; i++) {
                if (op.in[i] != t) continue;
                if (i == 0 && g.twin[c] >= 0 && !g.absorbed[c] && tw < 0) tw = c;
                else if (!(i == 0 && g.absorbed[c] && tw >= 0 && g.twin[tw] == c)) ok = 0;
            }
        }
        if (ok && tw >= 0) {
            g.planar[k] = 1;
            g.planar[tw] = 1;
        }
    }
}

// Sibling-fusion pass: in an HRModule fuse layer the branch-0 tensor (32 ch @ 64x48) is the
// input of up to three 3x3/s2 convs (-> 64 ch for branch 1; -> 32 ch + ReLU starting the
// chains to branches 2 and 3).  They run as ONE launch over cout-concatenated weights
// (s2conv_multi): the 201 MB input is read once instead of once per conv.
void sib_fuse(Graph& g, bool enable) {
    const int no = (int)g.ops.size();
    g.sib.assign(no, {});
    g.sib_w.assign(no, nullptr);
    g.t16_w.assign(no, nullptr);
    g.tr_w.assign(no, nullptr);
    g.sib_b.assign(no, nullptr);
    if (!enable) return;
    auto plain_s2 = [&](int k) {
        const mvp_op_desc& op = g.ops[k];
        return op.kind == MVP_OP_CONV && !g.absorbed[k] && !g.block_head[k] && g.cat_src[k] < 0 &&
               g.pair_tail[k] < 0 && g.stem_head[k] < 0 && g.twin[k] < 0 && op.ks == 3 && op.stride == 2 &&
               (op.n_in < 2 || op.in[1] < 0) && op.cout % 32 == 0 && g.tensors[op.out].dtype == MVP_DT_BF16_NHWC;
    };
    for (int a = 0; a < no; a++) {
        if (!plain_s2(a)) continue;
        const mvp_op_desc& A = g.ops[a];
        const mvp_tensor_desc& x = g.tensors[A.in[0]];
        int tot = A.cout;
        std::vector<int> list;
        for (int b = a + 1; b < no && list.size() < 2; b++) {
            const mvp_op_desc& B = g.ops[b];
            if (B.in[0] != A.in[0] || !plain_s2(b) || B.segment != A.segment) continue;
            if (!s2conv_multi_supported(x.h, x.w, x.c, tot + B.cout)) continue;
            list.push_back(b);
            tot += B.cout;
        }
        if (list.empty()) continue;
        for (int b : list) g.absorbed[b] = 1;
        g.sib[a] = list;
    }
}

// Head-fusion pass: the last fuse layer's out0 (32 ch @ 64x48) feeds only the heatmap head
// (1x1 32 -> 17, f32 NCHW); the head kernel forms out0 per pixel itself, so the 201 MB
// tensor is never written or re-read (bit-identical: same sums, same bf16 rounding).
void head_fuse(Graph& g, bool enable) {
    const int no = (int)g.ops.size(), nt = (int)g.tensors.size();
    g.head_src.assign(no, -1);
    if (!enable) return;
    std::vector<int> uses(nt, 0), producer(nt, -1);
    for (int k = 0; k < no; k++) {
        const mvp_op_desc& op = g.ops[k];
        producer[op.out] = k;
        for (int i = 0; i < op.n_in; i++)
            if (op.in[i] >= 0) uses[op.in[i]]++;
    }
    for (int k = 0; k < no; k++) {
        const mvp_op_desc& H = g.ops[k];
        if (H.kind != MVP_OP_CONV || g.absorbed[k] || g.tensors[H.out].dtype != MVP_DT_F32_NCHW || H.ks != 1 ||
            H.relu || (H.n_in > 1 && H.in[1] >= 0))
            continue;
        const int f = producer[H.in[0]];
        if (f < 0 || g.absorbed[f] || g.ops[f].kind != MVP_OP_FUSE || uses[H.in[0]] != 1 || H.in[0] == g.output ||
            g.ops[f].segment != H.segment)
            continue;
        if (!head_fuse_supported(H.cin, H.cout, g.ops[f].n_in)) continue;
        g.absorbed[f] = 1;
        g.head_src[k] = f;
    }
}

// Device-side concatenated weights / summed biases of the cat-fused ops: allocated at graph
// create time, filled from the blobs by cat_fill (create and mvp_graph_refresh_weights).
void cat_alloc(Graph& g) {
    for (int b = 0; b < (int)g.ops.size(); b++) {
        const int a = g.cat_src[b];
        if (a < 0) continue;
        const mvp_op_desc& B = g.ops[b];
        const int cp = conv_cout_pad(B.cout), cin = B.cin + g.ops[a].cin;
        MVP_HIP(hipMalloc(&g.cat_w[b], (size_t)cp * cin * sizeof(uint16_t)));
        MVP_HIP(hipMalloc(&g.cat_b[b], (size_t)cp * sizeof(float)));
    }
}

void sib_alloc(Graph& g) {
    for (int a = 0; a < (int)g.ops.size(); a++) {
        if (g.sib[a].empty()) continue;
        const int kk = 9 * g.ops[a].cin;
        MVP_HIP(hipMalloc(&g.sib_w[a], (size_t)128 * kk * sizeof(uint16_t)));
        MVP_HIP(hipMalloc(&g.sib_b[a], (size_t)128 * sizeof(float)));
    }
}

void sib_fill(Graph& g) {
    for (int a = 0; a < (int)g.ops.size(); a++) {
        if (g.sib[a].empty()) continue;
        const int kk = 9 * g.ops[a].cin;
        MVP_HIP(hipMemset(g.sib_w[a], 0, (size_t)128 * kk * sizeof(uint16_t)));
        MVP_HIP(hipMemset(g.sib_b[a], 0, (size_t)128 * sizeof(float)));
        int row = 0;
        std::vector<int> members{a};
        members.insert(members.end(), g.sib[a].begin(), g.sib[a].end());
        for (int m : members) {
            const mvp_op_desc& op = g.ops[m];
            MVP_HIP(hipMemcpy(g.sib_w[a] + (size_t)row * kk, g.wb + op.w_off, (size_t)op.cout * kk * sizeof(uint16_t),
                              hipMemcpyDeviceToDevice));
            MVP_HIP(hipMemcpy(g.sib_b[a] + row, g.fb + op.b_off, (size_t)op.cout * sizeof(float),
                              hipMemcpyDeviceToDevice));
            row += op.cout;
        }
    }
}

void cat_fill(Graph& g) {
    for (int b = 0; b < (int)g.ops.size(); b++) {
        const int a = g.cat_src[b];
        if (a < 0) continue;
        const mvp_op_desc& B = g.ops[b];
        const mvp_op_desc& A = g.ops[a];
        const int cp = conv_cout_pad(B.cout), cin = B.cin + A.cin;
        MVP_HIP(hipMemcpy2D(g.cat_w[b], (size_t)cin * 2, g.wb + B.w_off, (size_t)B.cin * 2, (size_t)B.cin * 2, cp,
                            hipMemcpyDeviceToDevice));
        MVP_HIP(hipMemcpy2D(g.cat_w[b] + B.cin, (size_t)cin * 2, g.wb + A.w_off, (size_t)A.cin * 2,
                            (size_t)A.cin * 2, cp, hipMemcpyDeviceToDevice));
        std::vector<float> hb(cp), ha(cp);
        MVP_HIP(hipMemcpy(hb.data(), g.fb + B.b_off, cp * sizeof(float), hipMemcpyDeviceToHost));
        MVP_HIP(hipMemcpy(ha.data(), g.fb + A.b_off, cp * sizeof(float), hipMemcpyDeviceToHost));
        for (int i = 0; i < cp; i++) hb[i] += ha[i];
        MVP_HIP(hipMemcpy(g.cat_b[b], hb.data(), cp * sizeof(float), hipMemcpyHostToDevice));
    }
}

// Weight images of the convs tconv16.hip serves (alloc at create, refilled with the blobs).
long t16_elems(const Graph& g, int k) {
    const mvp_op_desc& op = g.ops[k];
    if (op.kind != MVP_OP_CONV || g.absorbed[k] || g.cat_src[k] >= 0 || g.pair_tail[k] >= 0 || g.bneck[k] >= 0 ||
        (op.stride == 1 && !op.relu) || g.tensors[op.out].dtype == MVP_DT_F32_NCHW || !g.sib[k].empty() ||
        g.twin[k] >= 0 || g.stem_head[k] >= 0)
        return 0;
    const mvp_tensor_desc& x = g.tensors[op.in[0]];
    return tconv16_image_elems(op.cin, op.cout, x.h, x.w, op.ks, op.stride);
}

void t16_alloc(Graph& g) {
    for (int k = 0; k < (int)g.ops.size(); k++) {
        const long n = t16_elems(g, k);
        if (n > 0) MVP_HIP(hipMalloc(&g.t16_w[k], (size_t)n * sizeof(uint16_t)));
        if (g.twin[k] >= 0 && !g.absorbed[k]) MVP_HIP(hipMalloc(&g.tr_w[k], (size_t)kTrans1ImageElems * sizeof(uint16_t)));
    }
}

void t16_fill(Graph& g) {
    for (int k = 0; k < (int)g.ops.size(); k++) {
        if (g.t16_w[k]) tconv16_pack_weights(g.wb + g.ops[k].w_off, g.t16_w[k], g.ops[k].cin, g.ops[k].cout, nullptr);
        if (g.tr_w[k]) trans1_pack_weights(g.wb, g.ops[k].w_off, g.ops[g.twin[k]].w_off, g.tr_w[k], nullptr);
    }
    MVP_HIP(hipDeviceSynchronize());
}

void cat_free(Graph& g) {
    for (uint16_t* p : g.t16_w)
        if (p) (void)hipFree(p);
    for (uint16_t* p : g.tr_w)
        if (p) (void)hipFree(p);
    g.t16_w.clear();
    g.tr_w.clear();
    for (uint16_t* p : g.cat_w)
        if (p) (void)hipFree(p);
    for (float* p : g.cat_b)
        if (p) (void)hipFree(p);
    for (uint16_t* p : g.sib_w)
        if (p) (void)hipFree(p);
    for (float* p : g.sib_b)
        if (p) (void)hipFree(p);
    g.cat_w.clear();
    g.cat_b.clear();
    g.sib_w.clear();
    g.sib_b.clear();
}

// Greedy first-fit placement of tensors in one arena by lifetime [def, last use].
// A tensor produced and consumed only inside one micro-batched segment is
// "local": it is sized for one micro-batch and re-used by every micro-batch.
// Every other tensor a micro-batched segment touches is sliced per micro-batch,
// so its lifetime is widened to the whole segment (later micro-batches replay
// the segment's ops).
void plan(Graph& g) {
    const int nt = (int)g.tensors.size();
    const int no = (int)g.ops.size();
    std::vector<int> first(nt, -1), last(nt, -1);
    std::vector<int> seg_of_def(nt, -1);
    std::vector<int> multi_seg(nt, 0);  // used by more than one segment
    std::vector<int> use_seg(nt, -1);
    for (int k = 0; k < no; k++) {
        if (g.absorbed[k]) continue;  // its output lives only in the fused kernel's LDS
        const mvp_op_desc& op = g.ops[k];
        first[op.out] = k;
        if (last[op.out] < k) last[op.out] = k;
        seg_of_def[op.out] = op.segment;
        auto touch = [&](int t) {
            if (use_seg[t] < 0) use_seg[t] = op.segment;
            else if (use_seg[t] != op.segment) multi_seg[t] = 1;
        };
        touch(op.out);
        for (int i = 0; i < op.n_in; i++) {
            if (op.in[i] < 0 || (g.block_head[k] && i == 0)) continue;  // fused: conv1's output is LDS-only
            if (g.stem_head[k] >= 0 && i == 0) continue;                 // fused stem: LDS-only
            if (g.head_src[k] >= 0 && i == 0) continue;                  // fused head: never materialised
            if (g.cat_src[k] >= 0 && i == 1) continue;                  // cat-fused: never materialised
            if (g.bneck[k] >= 0 && i == 0) continue;                     // fused Bottleneck: LDS-only
            last[op.in[i]] = std::max(last[op.in[i]], k);
            touch(op.in[i]);
        }
        if (g.cat_src[k] >= 0) {  // the absorbed op's input is read here
            const int x = g.ops[g.cat_src[k]].in[0];
            last[x] = std::max(last[x], k);
            touch(x);
        }
        if (g.twin[k] >= 0) {  // the absorbed sibling's output is written here
            const int y2 = g.ops[g.twin[k]].out;
            first[y2] = k;
            if (last[y2] < k) last[y2] = k;
            seg_of_def[y2] = op.segment;
            touch(y2);
        }
        for (int b : g.sib[k]) {  // the absorbed siblings' outputs are written here
            const int y2 = g.ops[b].out;
            first[y2] = k;
            if (last[y2] < k) last[y2] = k;
            seg_of_def[y2] = op.segment;
            touch(y2);
        }
        if (g.stem_head[k] >= 0) {  // the absorbed stem's input is read here
            const int x = g.ops[g.stem_head[k]].in[0];
            last[x] = std::max(last[x], k);
            touch(x);
        }
        if (g.head_src[k] >= 0) {  // the absorbed fuse's inputs are read here
            const mvp_op_desc& f = g.ops[g.head_src[k]];
            for (int i = 0; i < f.n_in; i++) {
                last[f.in[i]] = std::max(last[f.in[i]], k);
                touch(f.in[i]);
            }
        }
        if (g.pair_tail[k] >= 0) {  // the absorbed successor's output is written here
            const int y2 = g.ops[g.pair_tail[k]].out;
            first[y2] = k;
            if (last[y2] < k) last[y2] = k;
            seg_of_def[y2] = op.segment;
            touch(y2);
        }
    }
    g.local_seg.assign(nt, -1);
    for (int t = 0; t < nt; t++) {
        if (t == g.input || t == g.output || first[t] < 0) continue;
        const int sg = seg_of_def[t];
        if (!multi_seg[t] && g.segs[sg].micro_batch > 0 && g.segs[sg].micro_batch < g.max_batch) g.local_seg[t] = sg;
    }
    for (int k = 0; k < no; k++) {
        if (g.absorbed[k]) continue;
        const mvp_op_desc& op = g.ops[k];
        const Segment& sg = g.segs[op.segment];
        if (sg.micro_batch <= 0 || sg.micro_batch >= g.max_batch) continue;
        auto widen = [&](int t) {
            if (t < 0 || g.local_seg[t] >= 0) return;
            first[t] = std::min(first[t] < 0 ? sg.first_op : first[t], sg.first_op);
            last[t] = std::max(last[t], sg.last_op);
        };
        widen(op.out);
        for (int i = 0; i < op.n_in; i++)
            if (!(g.block_head[k] && i == 0) && !(g.cat_src[k] >= 0 && i == 1) && !(g.stem_head[k] >= 0 && i == 0) &&
                !(g.head_src[k] >= 0 && i == 0) && !(g.bneck[k] >= 0 && i == 0))
                widen(op.in[i]);
        if (g.head_src[k] >= 0)
            for (int i = 0; i < g.ops[g.head_src[k]].n_in; i++) widen(g.ops[g.head_src[k]].in[i]);
        if (g.stem_head[k] >= 0) widen(g.ops[g.stem_head[k]].in[0]);
        if (g.twin[k] >= 0) widen(g.ops[g.twin[k]].out);
        for (int b : g.sib[k]) widen(g.ops[b].out);
        if (g.cat_src[k] >= 0) widen(g.ops[g.cat_src[k]].in[0]);
        if (g.pair_tail[k] >= 0) widen(g.ops[g.pair_tail[k]].out);
    }
    std::vector<int> order;
    for (int t = 0; t < nt; t++)
        if (t != g.input && t != g.output && first[t] >= 0) order.push_back(t);
    auto alloc_bytes = [&](int t) {
        const int b = g.local_seg[t] >= 0 ? g.segs[g.local_seg[t]].micro_batch : g.max_batch;
        return (tensor_bytes(g.tensors[t], b) + 255) / 256 * 256;
    };
    std::sort(order.begin(), order.end(), [&](int a, int b) { return alloc_bytes(a) > alloc_bytes(b); });
    g.offset.assign(nt, -1);
    struct Placed {
        int64_t off, size;
        int first, last;
    };
    std::vector<Placed> placed;
    int64_t top = 0;
    for (int t : order) {
        const int64_t size = alloc_bytes(t);
        std::vector<Placed> live;
        for (const Placed& p : placed)
            if (!(p.last < first[t] || last[t] < p.first)) live.push_back(p);
        std::sort(live.begin(), live.end(), [](const Placed& a, const Placed& b) { return a.off < b.off; });
        int64_t off = 0;
        for (const Placed& p : live) {
            if (off + size <= p.off) break;
            off = std::max(off, p.off + p.size);
        }
        placed.push_back({off, size, first[t], last[t]});
        g.offset[t] = off;
        top = std::max(top, off + size);
    }
    g.arena_bytes = top;
}

}  // namespace
}  // namespace mvp

using mvp::Graph;

extern "C" int mvp_graph_create(const mvp_tensor_desc* tensors, int n_tensors, const mvp_op_desc* ops, int n_ops,
                                const int* seg_micro_batch, int n_segments, int input_tensor, int output_tensor,
                                const uint16_t* w_dev, int64_t w_elems, const float* f_dev, int64_t f_elems,
                                int max_batch, void** handle_out) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(handle_out != nullptr, "mvp_graph_create: handle_out is NULL");
    *handle_out = nullptr;
    MVP_REQUIRE(tensors && n_tensors > 0 && ops && n_ops > 0, "mvp_graph_create: empty graph");
    MVP_REQUIRE(input_tensor >= 0 && input_tensor < n_tensors && output_tensor >= 0 && output_tensor < n_tensors &&
                    input_tensor != output_tensor,
                "mvp_graph_create: bad input/output tensor ids");
    MVP_REQUIRE(max_batch > 0, "mvp_graph_create: max_batch must be > 0");
    MVP_REQUIRE(seg_micro_batch && n_segments > 0, "mvp_graph_create: segments missing");
    Graph* g = new Graph();
    try {
        g->tensors.assign(tensors, tensors + n_tensors);
        g->ops.assign(ops, ops + n_ops);
        g->input = input_tensor;
        g->output = output_tensor;
        g->wb = w_dev;
        g->fb = f_dev;
        g->max_batch = max_batch;
        g->segs.resize(n_segments);
        for (int i = 0; i < n_segments; i++) {
            MVP_REQUIRE(seg_micro_batch[i] >= 0, "mvp_graph_create: negative micro-batch");
            g->segs[i].micro_batch = seg_micro_batch[i];
        }
        mvp::validate(*g, w_elems, f_elems);
        const char* nf = getenv("MVPOSE_NO_FUSE");  // diagnostics: run every conv on its own
        mvp::fuse(*g, !(nf && nf[0] == '1'));
        const char* nc = getenv("MVPOSE_NO_CATFUSE");  // diagnostics: keep the downsample conv separate
        mvp::cat_fuse(*g, !(nc && nc[0] == '1') && !(nf && nf[0] == '1'));
        const char* np = getenv("MVPOSE_NO_PAIRFUSE");  // diagnostics: keep conv3 / next conv1 apart
        const bool pair_on = !(np && np[0] == '1') && !(nf && nf[0] == '1');
        mvp::bneck_fuse(*g, !(nf && nf[0] == '1'), pair_on && mvp::conv1x1_pair_supported(64, 256, 64));
        mvp::pair_fuse(*g, pair_on);
        mvp::stem_fuse(*g, !(nf && nf[0] == '1'));
        mvp::twin_fuse(*g, !(nf && nf[0] == '1'));
        mvp::planar_fuse(*g);
        mvp::sib_fuse(*g, !(nf && nf[0] == '1'));
        mvp::head_fuse(*g, !(nf && nf[0] == '1'));
        mvp::cat_alloc(*g);
        mvp::sib_alloc(*g);
        mvp::cat_fill(*g);
        mvp::sib_fill(*g);
        mvp::t16_alloc(*g);
        mvp::t16_fill(*g);
        mvp::plan(*g);
        if (g->arena_bytes > 0) {
            hipError_t e = hipMalloc(&g->arena, g->arena_bytes);
            if (e != hipSuccess)
                mvp::fail(MVP_ERR_NOMEM, "mvp_graph_create: arena of %lld bytes: %s", (long long)g->arena_bytes,
                          hipGetErrorString(e));
        }
    } catch (...) {
        mvp::cat_free(*g);
        delete g;
        throw;
    }
    *handle_out = g;
    MVP_ABI_END
}

extern "C" int mvp_graph_forward(void* handle, const void* input_dev, int batch, void* output_dev, void* stream) {
    MVP_ABI_BEGIN
    Graph* g = static_cast<Graph*>(handle);
    MVP_REQUIRE(g != nullptr, "mvp_graph_forward: NULL handle");
    MVP_REQUIRE(batch >= 0 && batch <= g->max_batch, "mvp_graph_forward: batch %d exceeds max_batch %d", batch,
                g->max_batch);
    MVP_REQUIRE(input_dev && output_dev, "mvp_graph_forward: NULL input/output");
    if (batch == 0) return MVP_OK;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int64_t slice = 0;  // first crop of the current micro-batch
    auto ptr = [&](int t) -> void* {
        const mvp_tensor_desc& d = g->tensors[t];
        if (g->local_seg[t] >= 0) return g->arena + g->offset[t];
        char* base = t == g->input ? (char*)const_cast<void*>(input_dev)
                     : t == g->output ? (char*)output_dev
                                      : g->arena + g->offset[t];
        return base + slice * mvp::tensor_bytes(d, 1);
    };
    auto run_op = [&](int k, int nb) {
        const mvp_op_desc& op = g->ops[k];
        const mvp_tensor_desc& o = g->tensors[op.out];
        if (g->absorbed[k]) return;
        if (g->block_head[k]) {
            const mvp_op_desc& c1 = g->ops[k - 1];
            auto launch = c1.cin == 32 ? mvp::launch_basic_block_c32 : mvp::launch_tblock64;
            launch((const uint16_t*)ptr(op.in[1]), g->wb + c1.w_off, g->fb + c1.b_off, g->wb + op.w_off,
                   g->fb + op.b_off, (uint16_t*)ptr(op.out), nb, o.h, o.w, s);
            return;
        }
        if (g->twin[k] >= 0) {  // transition1: this 3x3/s1 conv and its 3x3/s2 sibling, one pass
            const mvp_op_desc& b = g->ops[g->twin[k]];
            mvp::launch_trans1((const uint16_t*)ptr(op.in[0]), g->wb, op.w_off, g->fb + op.b_off, b.w_off,
                               g->fb + b.b_off, (uint16_t*)ptr(op.out), (uint16_t*)ptr(b.out), nb, s, g->tr_w[k],
                               g->planar[k]);
            return;
        }
        if (!g->sib[k].empty()) {  // this 3x3/s2 conv and its siblings on the same input
            const mvp_tensor_desc& x = g->tensors[op.in[0]];
            mvp::S2Multi m;
            m.x = (const uint16_t*)ptr(op.in[0]);
            m.w = g->sib_w[k];
            m.bias = g->sib_b[k];
            m.N = nb;
            m.H = x.h;
            m.W = x.w;
            m.Cin = op.cin;
            std::vector<int> members{k};
            members.insert(members.end(), g->sib[k].begin(), g->sib[k].end());
            m.n_out = (int)members.size();
            for (int i = 0; i < m.n_out; i++) {
                const mvp_op_desc& o2 = g->ops[members[i]];
                m.y[i] = (uint16_t*)ptr(o2.out);
                m.cout[i] = o2.cout;
                m.relu[i] = o2.relu;
            }
            mvp::launch_s2conv_multi(m, s);
            return;
        }
        if (g->head_src[k] >= 0) {  // the last fuse layer's out0, formed per pixel by the head
            const mvp_op_desc& f = g->ops[g->head_src[k]];
            const mvp_tensor_desc& fo = g->tensors[f.out];
            const uint16_t* ins[4];
            for (int i = 0; i < f.n_in; i++) ins[i] = (const uint16_t*)ptr(f.in[i]);
            mvp::launch_head_fuse(ins, f.up, f.n_in, f.relu, g->wb + op.w_off, g->fb + op.b_off, (float*)ptr(op.out),
                                  nb, fo.h, fo.w, s);
            return;
        }
        if (g->bneck[k] >= 0) {  // the whole Bottleneck: conv1 + conv2 (absorbed) + this conv3
            const mvp_op_desc& a = g->ops[g->bneck[k]];
            const mvp_op_desc& c2 = g->ops[g->bneck_mid[k]];
            const bool lead = g->bneck_lead[k];
            const mvp_tensor_desc& x = g->tensors[a.in[0]];
            mvp::BneckLaunch bl;
            bl.x = (const uint16_t*)ptr(a.in[0]);
            bl.w1 = g->wb + a.w_off;
            bl.b1 = g->fb + a.b_off;
            bl.w2 = g->wb + c2.w_off;
            bl.b2 = g->fb + c2.b_off;
            bl.w3 = lead ? g->cat_w[k] : g->wb + op.w_off;
            bl.b3 = lead ? g->cat_b[k] : g->fb + op.b_off;
            bl.y = (uint16_t*)ptr(op.out);
            bl.N = nb;
            bl.H = x.h;
            bl.W = x.w;
            bl.perm = g->bneck_perm[k];
            bl.lead = lead;
            bl.planar = g->planar[k];
            mvp::launch_bneck(bl, s);
            return;
        }
        if (g->stem_head[k] >= 0) {  // stem conv1 + this conv2 in one launch
            const mvp_op_desc& st = g->ops[g->stem_head[k]];
            const mvp_tensor_desc& x = g->tensors[st.in[0]];
            mvp::launch_stem2((const uint16_t*)ptr(st.in[0]), g->fb + st.w_off, g->fb + st.b_off, g->wb + op.w_off,
                              g->fb + op.b_off, (uint16_t*)ptr(op.out), nb, x.h, x.w, s);
            return;
        }
        if (op.kind == MVP_OP_STEM) {
            const mvp_tensor_desc& x = g->tensors[op.in[0]];
            mvp::launch_stem((const uint16_t*)ptr(op.in[0]), g->fb + op.w_off, g->fb + op.b_off,
                             (uint16_t*)ptr(op.out), nb, x.h, x.w, s);
        } else if (op.kind == MVP_OP_CONV) {
            const mvp_tensor_desc& x = g->tensors[op.in[0]];
            mvp::ConvLaunch c{};
            c.x = (const uint16_t*)ptr(op.in[0]);
            c.w = g->wb + op.w_off;
            c.bias = g->fb + op.b_off;
            c.res = (op.n_in > 1 && op.in[1] >= 0) ? (const uint16_t*)ptr(op.in[1]) : nullptr;
            c.out_f32_nchw = o.dtype == MVP_DT_F32_NCHW;
            c.y = c.out_f32_nchw ? nullptr : (uint16_t*)ptr(op.out);
            c.yf = c.out_f32_nchw ? (float*)ptr(op.out) : nullptr;
            c.N = nb;
            c.H = x.h;
            c.W = x.w;
            c.Cin = op.cin;
            c.Cout = op.cout;
            c.ks = op.ks;
            c.stride = op.stride;
            c.relu = op.relu;
            c.w_img = g->t16_w[k];
            if (g->cat_src[k] >= 0) {  // cat-fused: [in[0], absorbed op's input] x [W | W_absorbed]
                const mvp_op_desc& a = g->ops[g->cat_src[k]];
                c.x2 = (const uint16_t*)ptr(a.in[0]);
                c.c1 = op.cin;
                c.Cin = op.cin + a.cin;
                c.w = g->cat_w[k];
                c.bias = g->cat_b[k];
                c.res = nullptr;
            }
            if (g->pair_tail[k] >= 0) {  // Bottleneck join: this conv + the next block's conv1
                const mvp_op_desc& b = g->ops[g->pair_tail[k]];
                mvp::PairLaunch pl;
                pl.x = c.x;
                pl.x2 = c.x2;
                pl.c1 = c.x2 ? c.c1 : c.Cin;
                pl.c2 = c.x2 ? c.Cin - c.c1 : 0;
                pl.w1 = c.w;
                pl.b1 = c.bias;
                pl.res = c.res;
                pl.y = c.y;
                pl.w2 = g->wb + b.w_off;
                pl.b2 = g->fb + b.b_off;
                pl.y2 = (uint16_t*)ptr(b.out);
                pl.n_pix = (long)nb * x.h * x.w;
                mvp::launch_conv1x1_pair(pl, s);
                return;
            }
            mvp::launch_conv(c, s);
        } else {
            const uint16_t* ins[4];
            for (int i = 0; i < op.n_in; i++) ins[i] = (const uint16_t*)ptr(op.in[i]);
            mvp::launch_fuse_sum(ins, op.up, op.n_in, (uint16_t*)ptr(op.out), nb, o.h, o.w, o.c, op.relu, s);
        }
    };
    for (const mvp::Segment& sg : g->segs) {
        if (sg.last_op < sg.first_op) continue;
        const int mb = (sg.micro_batch > 0 && sg.micro_batch < batch) ? sg.micro_batch : batch;
        for (int64_t b0 = 0; b0 < batch; b0 += mb) {
            slice = b0;
            const int nb = (int)std::min<int64_t>(mb, batch - b0);
            for (int k = sg.first_op; k <= sg.last_op; k++) run_op(k, nb);
        }
        slice = 0;
    }
    MVP_ABI_END
}

// Launch plan of one forward (diagnostics for tools/fwd_breakdown.py: pairs the kernel trace with
// the graph's MACs so each kernel family gets its FLOP and MFMA fraction).  One record per kernel
// launch, in launch order: {launching op, route, crops in the launch, MACs of every op it covers}.
// route: 1 fused BasicBlock, 2 transition twin, 3 s2 siblings, 4 head + fuse, 5 Bottleneck,
// 6 stem pair, 7 stem, 8 conv, 9 1x1 pair, 10 fuse sum.
namespace {
int64_t op_macs(const Graph& g, int k) {
    const mvp_op_desc& op = g.ops[k];
    if (op.kind != MVP_OP_CONV && op.kind != MVP_OP_STEM) return 0;
    const mvp_tensor_desc& o = g.tensors[op.out];
    const int cin = op.kind == MVP_OP_STEM ? 3 : op.cin;
    return (int64_t)o.h * o.w * op.cout * cin * op.ks * op.ks;
}
}  // namespace

extern "C" int mvp_graph_plan(void* handle, int batch, int64_t* rec_out, int max_records, int* n_records,
                              int64_t* covered_macs_out) {
    MVP_ABI_BEGIN
    Graph* g = static_cast<Graph*>(handle);
    MVP_REQUIRE(g && rec_out && n_records, "mvp_graph_plan: NULL pointer");
    MVP_REQUIRE(batch > 0 && batch <= g->max_batch, "mvp_graph_plan: batch %d", batch);
    const int no = (int)g->ops.size();
    std::vector<int> seen(no, 0);
    int n = 0;
    int64_t total = 0;
    for (const mvp::Segment& sg : g->segs) {
        if (sg.last_op < sg.first_op) continue;
        const int mb = (sg.micro_batch > 0 && sg.micro_batch < batch) ? sg.micro_batch : batch;
        for (int64_t b0 = 0; b0 < batch; b0 += mb) {
            const int nb = (int)std::min<int64_t>(mb, batch - b0);
            for (int k = sg.first_op; k <= sg.last_op; k++) {
                if (g->absorbed[k]) continue;
                const mvp_op_desc& op = g->ops[k];
                std::vector<int> cov{k};
                int route;
                if (g->block_head[k]) { route = 1; cov.push_back(k - 1); }
                else if (g->twin[k] >= 0) { route = 2; cov.push_back(g->twin[k]); }
                else if (!g->sib[k].empty()) { route = 3; cov.insert(cov.end(), g->sib[k].begin(), g->sib[k].end()); }
                else if (g->head_src[k] >= 0) { route = 4; cov.push_back(g->head_src[k]); }
                else if (g->bneck[k] >= 0) {
                    route = 5;
                    cov.push_back(g->bneck[k]);
                    cov.push_back(g->bneck_mid[k]);
                    if (g->cat_src[k] >= 0) cov.push_back(g->cat_src[k]);
                }
                else if (g->stem_head[k] >= 0) { route = 6; cov.push_back(g->stem_head[k]); }
                else if (op.kind == MVP_OP_STEM) route = 7;
                else if (op.kind == MVP_OP_CONV) {
                    route = g->pair_tail[k] >= 0 ? 9 : 8;
                    if (g->cat_src[k] >= 0) cov.push_back(g->cat_src[k]);
                    if (g->pair_tail[k] >= 0) cov.push_back(g->pair_tail[k]);
                } else route = 10;
                int64_t macs = 0;
                for (int c : cov) {
                    macs += op_macs(*g, c);
                    if (b0 == 0) seen[c]++;
                }
                macs *= nb;
                total += macs;
                if (n < max_records) {
                    rec_out[4 * n + 0] = k;
                    rec_out[4 * n + 1] = route;
                    rec_out[4 * n + 2] = nb;
                    rec_out[4 * n + 3] = macs;
                }
                n++;
            }
        }
    }
    for (int k = 0; k < no; k++)
        MVP_REQUIRE(seen[k] == 1, "mvp_graph_plan: op %d covered by %d launches", k, seen[k]);
    *n_records = n;
    if (covered_macs_out) *covered_macs_out = total;
    MVP_ABI_END
}

// The blobs were rewritten in place (e.g. a weight broadcast from rank 0 after the graph was
// built): re-derive every weight the graph copied out of them at create time.  Blocking.
extern "C" int mvp_graph_refresh_weights(void* handle) {
    MVP_ABI_BEGIN
    Graph* g = static_cast<Graph*>(handle);
    MVP_REQUIRE(g != nullptr, "mvp_graph_refresh_weights: NULL handle");
    MVP_HIP(hipDeviceSynchronize());
    mvp::cat_fill(*g);
    mvp::sib_fill(*g);
    mvp::t16_fill(*g);
    MVP_HIP(hipDeviceSynchronize());
    MVP_ABI_END
}

extern "C" int mvp_graph_arena_bytes(void* handle, int64_t* bytes_out) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(handle && bytes_out, "mvp_graph_arena_bytes: NULL argument");
    *bytes_out = static_cast<Graph*>(handle)->arena_bytes;
    MVP_ABI_END
}

extern "C" int mvp_graph_destroy(void* handle) {
    MVP_ABI_BEGIN
    Graph* g = static_cast<Graph*>(handle);
    if (g) {
        if (g->arena) (void)hipFree(g->arena);
        mvp::cat_free(*g);
        delete g;
    }
    MVP_ABI_END
}
