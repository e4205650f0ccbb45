"""GPU parity of the branch-plane BasicBlock convolutions against a torch fp32
restatement that rounds to bf16 at the same tensor boundaries as the device
graph (bf16 weights and activations, f32 bias and accumulation).  Every conv
kernel family that serves a plane is checked: the generic conv_mfma_kernel
(conv.hip; block.hip for the fused 32-channel block), the 32x32x16 tconv.hip and
tconv16.hip.  They sum K in different orders, so each
is compared against the reference with a tolerance, not bit for bit:
  relative L2 error <= 4e-3, and |dev - ref| <= 3 bf16 ulps of max|ref|."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

PLANES = [(32, 64, 48), (64, 32, 24), (128, 16, 12), (256, 8, 6), (64, 64, 48)]
# environment per kernel family: the 32-channel plane runs the fused block,
# basic_block_c32_kernel ("generic") or tblock ("tconv"); the 64-channel plane at
# 32x24 runs tblock64 in "tconv" mode
_OFF = {"MVPOSE_NO_TCONV": "1", "MVPOSE_NO_TBLOCK": "1"}
MODES = {
    "generic": dict(_OFF),
    "tconv": dict(_OFF, MVPOSE_NO_TCONV="0", MVPOSE_NO_TBLOCK="0"),
    # tconv.hip's 64-cout tiles on the 128- and 256-channel planes (tconv16.hip by default)
    "tconv64": dict(_OFF, MVPOSE_NO_TCONV="0", MVPOSE_NO_TBLOCK="0", MVPOSE_TCONV16="0"),
}


def _bf(t):
    return t.to(torch.bfloat16).float()


def _reference(sd, x, n_blocks):
    """x: (N,H,W,C) bf16-valued f32 -> (N,H,W,C) bf16-valued f32."""
    from mvpose import hrnet
    y = x.permute(0, 3, 1, 2)
    for k in range(n_blocks):
        inp = y
        for j in (1, 2):
            w, b = hrnet.fold_bn(sd, f"b{k}.conv{j}", f"b{k}.bn{j}")
            wt = _bf(torch.from_numpy(np.ascontiguousarray(w.transpose(0, 3, 1, 2))).float())
            z = torch.nn.functional.conv2d(y, wt, padding=1) + torch.from_numpy(b).float()[None, :, None, None]
            if j == 2:
                z = z + inp
            y = _bf(torch.relu(z))
    return y.permute(0, 2, 3, 1).contiguous()


def _set_mode(monkeypatch, mode):
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)
    if mode != "tconv64":
        monkeypatch.delenv("MVPOSE_TCONV16", raising=False)


def _run(c, h, w, n, n_blocks, seed, monkeypatch, mode):
    from mvpose import hrnet
    _set_mode(monkeypatch, mode)
    spec, xi, yo, sd = hrnet.basic_block_spec(c, h, w, seed=seed, n_blocks=n_blocks)
    g = hrnet.ConvGraph(spec, xi, yo, max_batch=n)
    gen = torch.Generator().manual_seed(seed + 100)
    x = torch.randn((n, h, w, c), generator=gen).bfloat16()
    out = torch.empty_like(x).cuda()
    g.run(x.cuda(), out)
    torch.cuda.synchronize()
    g.close()
    return out.float().cpu(), _reference(sd, x.float(), n_blocks)


@pytest.mark.parametrize("c,h,w", PLANES)
def test_basic_block_vs_reference(c, h, w, monkeypatch):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    n = 37  # ragged: not a multiple of any tile / grid size
    for mode in MODES:
        got, ref = _run(c, h, w, n, 2, 3, monkeypatch, mode)
        assert torch.isfinite(got).all()
        rel = (torch.linalg.vector_norm(got - ref) / torch.linalg.vector_norm(ref)).item()
        mx = (got - ref).abs().max().item()
        scale = ref.abs().max().item()
        print(f"C={c} {h}x{w} {mode}: rel L2 {rel:.2e}, max abs {mx:.3e} (max|ref| {scale:.2f})")
        assert rel <= 4e-3
        assert mx <= 3 * scale * 2.0 ** -8


@pytest.mark.parametrize("stream", ["1", "0"])
@pytest.mark.parametrize("n", [1, 5, 37, 301])
def test_tblock64_bitwise_equals_two_tconv_launches(n, stream, monkeypatch):
    """The fused 64-channel BasicBlock (tblock64.hip: warp-specialised conv1 / conv2 waves,
    the intermediate only in LDS, a crop's tiles walked top to bottom with intermediate rows
    0-1 of tiles 1-3 copied from the previous tile) reproduces the two separate tconv launches
    bit for bit — same MFMA sequence per accumulator, same epilogues.  n = 1, 5, 37: one crop
    per workgroup; n = 301: more crops than CUs (ragged 1-2 crops per workgroup).
    stream = "1" forces the crop-contiguous ranges at every batch; "0" leaves the launcher's
    rule (conv.h crop_ranges_balanced), which below one crop per CU (n = 1, 5, 37) picks the
    strided mode: one tile per workgroup slot, no row reuse."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import hrnet
    _set_mode(monkeypatch, "tconv")
    monkeypatch.setenv("MVPOSE_CROP_STREAM", stream)
    spec, xi, yo, _ = hrnet.basic_block_spec(64, 32, 24, seed=13, n_blocks=2)
    gen = torch.Generator().manual_seed(14)
    x = torch.randn((n, 32, 24, 64), generator=gen).bfloat16().cuda()
    outs = []
    for off in ("1", "0"):
        monkeypatch.setenv("MVPOSE_NO_TBLOCK64", off)
        g = hrnet.ConvGraph(spec, xi, yo, max_batch=n)
        out = torch.empty_like(x)
        g.run(x, out)
        torch.cuda.synchronize()
        outs.append((out, g.arena_bytes))
        g.close()
    (a, arena_a), (b, arena_b) = outs
    d = (a.float() - b.float()).abs()
    print(f"tblock64 n={n}: max |fused - unfused| {d.max().item():.3g}, identical {(d == 0).float().mean().item():.6f}, "
          f"arena {arena_b} vs {arena_a}")
    assert torch.equal(a, b)
    assert arena_b < arena_a


@pytest.mark.parametrize("n", [1, 5, 37, 301, 700])
def test_tblock32s_bitwise_equals_tile_kernel(n, monkeypatch):
    """The streaming 32-channel BasicBlock (tblock32s.hip: whole crops per workgroup, input rows
    through a 30-row LDS ring, warp-specialised conv1 / conv2) reproduces the tile kernel
    (tblock.hip) bit for bit — same MFMA sequence per accumulator, same epilogues.  n = 1, 5,
    37: fewer crops than CUs (one crop per workgroup, unused CUs); 301, 700: ragged
    multi-crop ranges, so the ring wraps across crop boundaries."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import hrnet
    _set_mode(monkeypatch, "tconv")
    # Force the streaming kernel at these unbalanced batches (the launcher would pick the tile kernel).
    monkeypatch.setenv("MVPOSE_CROP_STREAM", "1")
    spec, xi, yo, _ = hrnet.basic_block_spec(32, 64, 48, seed=17, n_blocks=2)
    gen = torch.Generator().manual_seed(18)
    x = torch.randn((n, 64, 48, 32), generator=gen).bfloat16().cuda()
    outs = []
    for off in ("1", "0"):
        monkeypatch.setenv("MVPOSE_NO_TBLOCK32S", off)
        g = hrnet.ConvGraph(spec, xi, yo, max_batch=n)
        out = torch.full_like(x, float("nan"))
        g.run(x, out)
        torch.cuda.synchronize()
        outs.append(out)
        g.close()
    a, b = outs
    d = (a.float() - b.float()).abs()
    print(f"tblock32s n={n}: max |stream - tile| {d.max().item():.3g}, identical {(d == 0).float().mean().item():.6f}")
    assert torch.equal(a, b)


@pytest.mark.parametrize("c,h,w,n", [(128, 16, 12, 1), (128, 16, 12, 1100), (256, 8, 6, 5), (256, 8, 6, 2100)])
def test_tconv16_tile_ranges_vs_reference(c, h, w, n, monkeypatch):
    """tconv16.hip at batch sizes the 37-crop test does not reach: one crop (a single tile,
    seven empty XCD slots of its group of 8), and batches whose tiles outnumber the CUs so
    that each workgroup loops over several tiles (2100 crops of the 256-ch plane: its two
    128-cout blocks on a fixed cout block per workgroup, XCD-major tile order)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    got, ref = _run(c, h, w, n, 1, 21, monkeypatch, "tconv")
    assert torch.isfinite(got).all()
    rel = (torch.linalg.vector_norm(got - ref) / torch.linalg.vector_norm(ref)).item()
    mx = (got - ref).abs().max().item()
    scale = ref.abs().max().item()
    print(f"tconv16 C={c} {h}x{w} n={n}: rel L2 {rel:.2e}, max abs {mx:.3e} (max|ref| {scale:.2f})")
    assert rel <= 4e-3
    assert mx <= 3 * scale * 2.0 ** -8


@pytest.mark.parametrize("mode", ["generic", "tconv", "tconv64"])
@pytest.mark.parametrize("c,h,w", [(32, 64, 48), (64, 32, 24), (128, 16, 12), (256, 8, 6)])
def test_batch_positions(c, h, w, mode, monkeypatch):
    """A crop's output must not depend on its batch position or the batch size
    (tile scheduling over a persistent grid, multi-crop tiles)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import hrnet
    _set_mode(monkeypatch, mode)
    spec, xi, yo, _ = hrnet.basic_block_spec(c, h, w, seed=5)
    g = hrnet.ConvGraph(spec, xi, yo, max_batch=600)
    gen = torch.Generator().manual_seed(9)
    x = torch.randn((600, h, w, c), generator=gen).bfloat16().cuda()
    full = torch.empty_like(x)
    g.run(x, full)
    part = torch.empty_like(x[:3])
    g.run(x[411:414].contiguous(), part)
    torch.cuda.synchronize()
    g.close()
    assert torch.equal(full[411:414], part)


@pytest.mark.parametrize("cin,cout,h,w,k", [(64, 256, 64, 48, 1), (256, 64, 64, 48, 1), (64, 64, 64, 48, 1),
                                            (64, 32, 32, 24, 1), (128, 64, 16, 12, 1), (256, 128, 8, 6, 1),
                                            (256, 32, 64, 48, 3)])
def test_projection_vs_reference(cin, cout, h, w, k):
    """y = relu(conv_b(x) + conv_a(x)): 1x1 convs (conv1x1.hip, permuted-cout epilogue) and
    transition1's 256->32 3x3 (tconv.hip with 32-cout tiles for conv_b)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import hrnet
    spec, xi, yo, sd = hrnet.projection_spec(cin, cout, h, w, k=k, seed=4)
    n = 23
    g = hrnet.ConvGraph(spec, xi, yo, max_batch=n)
    gen = torch.Generator().manual_seed(8)
    x = torch.randn((n, h, w, cin), generator=gen).bfloat16()
    out = torch.empty((n, h, w, cout), dtype=torch.bfloat16, device="cuda")
    g.run(x.cuda(), out)
    torch.cuda.synchronize()
    g.close()
    xf = x.float().permute(0, 3, 1, 2)
    zs = []
    for j in ("a", "b"):
        wt, b = hrnet.fold_bn(sd, j, f"{j}bn")
        wt = _bf(torch.from_numpy(np.ascontiguousarray(wt.transpose(0, 3, 1, 2))).float())
        zs.append(torch.nn.functional.conv2d(xf, wt, padding=k // 2) + torch.from_numpy(b).float()[None, :, None, None])
    t = _bf(zs[0])
    ref = _bf(torch.relu(zs[1] + t)).permute(0, 2, 3, 1)
    got = out.float().cpu()
    rel = (torch.linalg.vector_norm(got - ref) / torch.linalg.vector_norm(ref)).item()
    mx = (got - ref).abs().max().item()
    print(f"{k}x{k} {cin}->{cout} {h}x{w}: rel L2 {rel:.2e}, max abs {mx:.3e}")
    assert rel <= 4e-3 and mx <= 3 * ref.abs().max().item() * 2.0 ** -8


@pytest.mark.parametrize("cat", [False, True])
@pytest.mark.parametrize("pair", [False, True])
def test_bottleneck_join(cat, pair, monkeypatch):
    """Layer1 conv3 (+ residual, or + the cat-fused downsample) followed by the next
    block's 256 -> 64 conv1, with the pair-fusion pass on (one conv1x1_pair launch,
    the second GEMM's K order permuted) and off (two conv1x1 launches), against a
    torch fp32 restatement with bf16 rounding at the graph's tensor boundaries."""
    from mvpose import hrnet
    monkeypatch.setenv("MVPOSE_NO_PAIRFUSE", "0" if pair else "1")
    h, w, n = 64, 48, 3
    spec, xi, yo, sd = hrnet.join_spec(h, w, seed=21, cat=cat)
    g = hrnet.ConvGraph(spec, xi, yo, max_batch=n)
    gen = torch.Generator().manual_seed(22)
    x = torch.randn((n, h, w, 64), generator=gen).bfloat16()
    out = torch.empty((n, h, w, 64), dtype=torch.bfloat16, device="cuda")
    g.run(x.cuda(), out)
    torch.cuda.synchronize()

    def conv(name, t):
        wt, b = hrnet.fold_bn(sd, name, name + "bn")
        wt = _bf(torch.from_numpy(np.ascontiguousarray(wt.transpose(0, 3, 1, 2))).float())
        return torch.nn.functional.conv2d(t, wt) + torch.from_numpy(b).float()[None, :, None, None]

    xf = x.float().permute(0, 3, 1, 2)
    r = conv("r", xf)
    r = r if cat else _bf(torch.relu(r))
    y = _bf(torch.relu(conv("a", xf) + r))
    ref = _bf(torch.relu(conv("b", y))).permute(0, 2, 3, 1)
    dev = out.float().cpu()
    rel = (torch.linalg.vector_norm(dev - ref) / torch.linalg.vector_norm(ref)).item()
    assert rel <= 4e-3, rel
    ulp = 2.0 ** (torch.floor(torch.log2(ref.abs().max())) - 7)
    assert (dev - ref).abs().max().item() <= 3 * ulp, ((dev - ref).abs().max().item(), ulp)


@pytest.mark.parametrize("n", [1, 5, 13, 300])
def test_stem2_streaming_bitwise_equals_tile_kernel(n, monkeypatch):
    """The streaming stem2 kernel (conv1 rows in a ring, warp-specialised conv1 / conv2 waves,
    one workgroup per crop range) against the tile kernel (MVPOSE_STEM2_TILE=1): same K order
    and MFMA sequence per output, so bit-identical; n covers one crop per workgroup, ragged
    ranges and more crops than CUs."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import hrnet
    # Force the streaming kernel at these unbalanced batches (the launcher would pick the tile kernel).
    monkeypatch.setenv("MVPOSE_CROP_STREAM", "1")
    spec, xi, yo, sd = hrnet.stem_spec(seed=33)
    gen = torch.Generator().manual_seed(34)
    x = torch.zeros((n, 256, 192, 4))
    x[..., :3] = torch.randn((n, 256, 192, 3), generator=gen)
    xb = x.bfloat16().cuda()
    outs = {}
    for tile in ("1", "0"):
        monkeypatch.setenv("MVPOSE_STEM2_TILE", tile)
        g = hrnet.ConvGraph(spec, xi, yo, max_batch=n)
        out = torch.full((n, 64, 48, 64), float("nan"), dtype=torch.bfloat16, device="cuda")
        g.run(xb, out)
        torch.cuda.synchronize()
        g.close()
        outs[tile] = out.cpu()
    assert torch.isfinite(outs["0"].float()).all()
    assert torch.equal(outs["0"].view(torch.int16), outs["1"].view(torch.int16))


@pytest.mark.parametrize("fused", [False, True])
def test_stem_vs_reference(fused, monkeypatch):
    """HRNet stem conv1 (3x3/s2, 4 -> 64) + conv2 (3x3/s2, 64 -> 64): the fused stem2.hip
    launch (conv1's 128x96x64 output only in LDS) and the two-launch path, against a
    torch fp32 restatement with bf16 weights and a bf16 conv1 output (the graph's
    rounding points); ragged batch."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import hrnet
    monkeypatch.setenv("MVPOSE_NO_STEMFUSE", "0" if fused else "1")
    spec, xi, yo, sd = hrnet.stem_spec(seed=31)
    n = 13
    g = hrnet.ConvGraph(spec, xi, yo, max_batch=n)
    gen = torch.Generator().manual_seed(32)
    x = torch.zeros((n, 256, 192, 4))
    x[..., :3] = torch.randn((n, 256, 192, 3), generator=gen)
    xb = x.bfloat16()
    out = torch.empty((n, 64, 48, 64), dtype=torch.bfloat16, device="cuda")
    g.run(xb.cuda(), out)
    torch.cuda.synchronize()
    arena = g.arena_bytes
    g.close()

    def conv(name, bn, t):
        wt, b = hrnet.fold_bn(sd, name, bn)
        wt = _bf(torch.from_numpy(np.ascontiguousarray(wt.transpose(0, 3, 1, 2))).float())
        return torch.nn.functional.conv2d(t, wt, stride=2, padding=1) + torch.from_numpy(b).float()[None, :, None, None]

    xf = xb.float()[..., :3].permute(0, 3, 1, 2)
    h = _bf(torch.relu(conv("backbone.conv1", "backbone.bn1", xf)))
    ref = _bf(torch.relu(conv("backbone.conv2", "backbone.bn2", h))).permute(0, 2, 3, 1)
    dev = out.float().cpu()
    rel = (torch.linalg.vector_norm(dev - ref) / torch.linalg.vector_norm(ref)).item()
    mx = (dev - ref).abs().max().item()
    print(f"stem fused={fused}: rel L2 {rel:.2e}, max abs {mx:.3e}, arena {arena}")
    assert rel <= 4e-3 and mx <= 3 * ref.abs().max().item() * 2.0 ** -8
    if fused:
        assert arena == 0  # the 128x96x64 intermediate is never allocated


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("output", [0, 1])
def test_transition1_vs_reference(fused, output, monkeypatch):
    """HRNet transition1 on the layer1 output: t0 (3x3/s1 256 -> 32) and t1 (3x3/s2 256 -> 64)
    from one pass over the 256-ch tensor (trans1.hip) and as two launches, against a torch
    fp32 restatement with bf16 weights; ragged batch."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import hrnet
    monkeypatch.setenv("MVPOSE_NO_TRANSFUSE", "0" if fused else "1")
    spec, xi, yo, sd = hrnet.transition_spec(seed=51, output=output)
    n = 11
    g = hrnet.ConvGraph(spec, xi, yo, max_batch=n)
    gen = torch.Generator().manual_seed(52)
    x = torch.relu(torch.randn((n, 64, 48, 256), generator=gen)).bfloat16()
    ho, wo, co = spec.tensors[yo][:3]
    out = torch.empty((n, ho, wo, co), dtype=torch.bfloat16, device="cuda")
    g.run(x.cuda(), out)
    torch.cuda.synchronize()
    g.close()
    name = ("t0", "t1")[output]
    wt, b = hrnet.fold_bn(sd, name, name + "bn")
    wt = _bf(torch.from_numpy(np.ascontiguousarray(wt.transpose(0, 3, 1, 2))).float())
    z = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), wt, stride=1 + output, padding=1)
    ref = _bf(torch.relu(z + torch.from_numpy(b).float()[None, :, None, None])).permute(0, 2, 3, 1)
    dev = out.float().cpu()
    rel = (torch.linalg.vector_norm(dev - ref) / torch.linalg.vector_norm(ref)).item()
    mx = (dev - ref).abs().max().item()
    print(f"transition1 t{output} fused={fused}: rel L2 {rel:.2e}, max abs {mx:.3e}")
    assert rel <= 4e-3 and mx <= 3 * ref.abs().max().item() * 2.0 ** -8


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("n_sib,output", [(3, 0), (3, 1), (3, 2), (2, 0), (2, 1)])
def test_fuse_layer_siblings_vs_reference(fused, n_sib, output, monkeypatch):
    """A fuse layer's 3x3/s2 convs on the branch-0 tensor (-> 64 no ReLU, -> 32 ReLU, -> 32
    ReLU; stage 3 has the first two): one launch over cout-concatenated weights
    (s2conv_multi, graph sibling fusion) and one launch each, against a torch fp32
    restatement with bf16 weights; ragged batch."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import hrnet
    monkeypatch.setenv("MVPOSE_NO_SIBFUSE", "0" if fused else "1")
    spec, xi, yo, sd = hrnet.sibling_spec(seed=61 + n_sib, output=output, n=n_sib)
    n = 9
    g = hrnet.ConvGraph(spec, xi, yo, max_batch=n)
    gen = torch.Generator().manual_seed(62)
    x = torch.relu(torch.randn((n, 64, 48, 32), generator=gen)).bfloat16()
    ho, wo, co = spec.tensors[yo][:3]
    out = torch.empty((n, ho, wo, co), dtype=torch.bfloat16, device="cuda")
    g.run(x.cuda(), out)
    torch.cuda.synchronize()
    g.close()
    name, _, relu = hrnet.SIBLINGS[output]
    wt, b = hrnet.fold_bn(sd, name, name + "bn")
    wt = _bf(torch.from_numpy(np.ascontiguousarray(wt.transpose(0, 3, 1, 2))).float())
    z = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), wt, stride=2, padding=1)
    z = z + torch.from_numpy(b).float()[None, :, None, None]
    ref = _bf(torch.relu(z) if relu else z).permute(0, 2, 3, 1)
    dev = out.float().cpu()
    rel = (torch.linalg.vector_norm(dev - ref) / torch.linalg.vector_norm(ref)).item()
    mx = (dev - ref).abs().max().item()
    assert rel <= 4e-3 and mx <= 3 * ref.abs().max().item() * 2.0 ** -8, (rel, mx)
