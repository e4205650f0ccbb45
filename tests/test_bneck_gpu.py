"""The streaming fused Bottleneck (csrc/bneck.hip) on HRNet-W32's layer1 plane (256 ch @ 64x48):
conv1 (1x1 -> 64), conv2 (3x3), conv3 (1x1 -> 256) + identity in one launch, the two 64-ch
intermediates only in LDS.  Against the unfused graph (MVPOSE_NO_BNECK=1: the 1x1 / Bottleneck
join kernels and the 3x3 tconv) it must be bit-identical — it reproduces each conv's MFMA
sequence and epilogue (conv1 in the join's permuted K order when the graph would have joined it
to the previous block, the 1x1 kernel's otherwise) — and it must match a torch fp32 restatement
(bf16 weights, bf16 rounding at the graph's tensor boundaries) to bf16 tolerance."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _bf(t):
    return t.to(torch.bfloat16).float()


def _run(spec, xi, yo, x, monkeypatch, fused):
    from mvpose import hrnet
    monkeypatch.setenv("MVPOSE_NO_BNECK", "0" if fused else "1")
    g = hrnet.ConvGraph(spec, xi, yo, max_batch=x.shape[0])
    out = torch.full((x.shape[0], 64, 48, 256), float("nan"), dtype=torch.bfloat16, device="cuda")
    g.run(x, out)
    torch.cuda.synchronize()
    arena = g.arena_bytes
    g.close()
    return out, arena


@pytest.mark.parametrize("n", [1, 5, 37, 300])
def test_layer1_bitwise_equals_unfused(n, monkeypatch):
    """HRNet's layer1 (block 0 with its downsample, then three fused Bottlenecks whose conv1 the
    unfused graph runs inside the previous block's join): n = 1, 5, 37 give one crop per
    workgroup; 300 gives ragged 1-2 crop ranges, so the x ring wraps across crop boundaries."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import hrnet
    spec, xi, yo, _ = hrnet.bottleneck_spec(seed=71, n_blocks=4, lead=True)
    gen = torch.Generator().manual_seed(72)
    x = torch.relu(torch.randn((n, 64, 48, 64), generator=gen)).bfloat16().cuda()
    a, arena_a = _run(spec, xi, yo, x, monkeypatch, False)
    b, arena_b = _run(spec, xi, yo, x, monkeypatch, True)
    d = (a.float() - b.float()).abs()
    print(f"layer1 n={n}: max |fused - unfused| {d.max().item():.3g}, identical "
          f"{(d == 0).float().mean().item():.6f}, arena {arena_b} vs {arena_a}")
    assert torch.isfinite(b.float()).all()
    assert torch.equal(a.view(torch.int16), b.view(torch.int16))
    assert arena_b < arena_a


def test_bneck_plain_order_bitwise_equals_unfused(monkeypatch):
    """A 256-ch input: the first block's conv1 has no join in front of it (the unfused graph runs
    it as a plain 1x1 conv, natural K order), the second's is joined (permuted order)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import hrnet
    spec, xi, yo, _ = hrnet.bottleneck_spec(seed=73, n_blocks=2, lead=False)
    gen = torch.Generator().manual_seed(74)
    x = torch.relu(torch.randn((9, 64, 48, 256), generator=gen)).bfloat16().cuda()
    a, _ = _run(spec, xi, yo, x, monkeypatch, False)
    b, _ = _run(spec, xi, yo, x, monkeypatch, True)
    assert torch.isfinite(b.float()).all()
    assert torch.equal(a.view(torch.int16), b.view(torch.int16))


def test_bneck_vs_reference(monkeypatch):
    """One fused Bottleneck against a torch fp32 restatement: relative L2 <= 4e-3 and
    |dev - ref| <= 3 bf16 ulps of max|ref| (the conv kernels' K orders differ from torch's)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import hrnet
    spec, xi, yo, sd = hrnet.bottleneck_spec(seed=75, n_blocks=1, lead=False)
    n = 7
    gen = torch.Generator().manual_seed(76)
    x = torch.relu(torch.randn((n, 64, 48, 256), generator=gen)).bfloat16()
    out, _ = _run(spec, xi, yo, x.cuda(), monkeypatch, True)

    def conv(name, t, k):
        w, b = hrnet.fold_bn(sd, name, name + "bn")
        wt = _bf(torch.from_numpy(np.ascontiguousarray(w.transpose(0, 3, 1, 2))).float())
        return torch.nn.functional.conv2d(t, wt, padding=k // 2) + torch.from_numpy(b).float()[None, :, None, None]

    xf = x.float().permute(0, 3, 1, 2)
    t1 = _bf(torch.relu(conv("b0.conv1", xf, 1)))
    t2 = _bf(torch.relu(conv("b0.conv2", t1, 3)))
    ref = _bf(torch.relu(conv("b0.conv3", t2, 1) + xf)).permute(0, 2, 3, 1)
    dev = out.float().cpu()
    rel = (torch.linalg.vector_norm(dev - ref) / torch.linalg.vector_norm(ref)).item()
    mx = (dev - ref).abs().max().item()
    print(f"bneck vs torch: rel L2 {rel:.2e}, max abs {mx:.3e} (max|ref| {ref.abs().max().item():.2f})")
    assert rel <= 4e-3 and mx <= 3 * ref.abs().max().item() * 2.0 ** -8


@pytest.mark.parametrize("output", [0, 1])
@pytest.mark.parametrize("n", [3, 300])
def test_layer1_transition_planar_bitwise_equals_unfused(output, n, monkeypatch):
    """Layer1 + transition1: with the fusion on, the last Bottleneck writes its output in
    chunk-planar layout and trans1 reads it so (graph planar pass); t0 / t1 must equal the
    unfused graph's (NHWC hand-off) bit for bit."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import hrnet
    spec, xi, yo, _ = hrnet.layer1_transition_spec(seed=81, output=output)
    ho, wo, co = spec.tensors[yo][:3]
    gen = torch.Generator().manual_seed(82)
    x = torch.relu(torch.randn((n, 64, 48, 64), generator=gen)).bfloat16().cuda()
    outs = []
    for fused in (False, True):
        monkeypatch.setenv("MVPOSE_NO_BNECK", "0" if fused else "1")
        g = hrnet.ConvGraph(spec, xi, yo, max_batch=n)
        out = torch.full((n, ho, wo, co), float("nan"), dtype=torch.bfloat16, device="cuda")
        g.run(x, out)
        torch.cuda.synchronize()
        g.close()
        outs.append(out)
    assert torch.isfinite(outs[1].float()).all()
    assert torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16))
