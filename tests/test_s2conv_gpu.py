"""GPU parity of the 3x3/stride-2 convolutions (s2conv.hip, polyphase halo) against
a torch fp32 restatement with bf16 weights/activations, on every stride-2 plane of
HRNet-W32, with and without ReLU, at batch sizes that leave partial crop groups
(NB = 2 and 4 crops per tile).  The generic conv_mfma_kernel path
(MVPOSE_NO_S2CONV=1) is checked against the same reference.  Tolerance as the
other conv tests: relative L2 <= 4e-3 and |dev - ref| <= 3 bf16 ulps of max|ref|."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

# (cin, cout, input h, input w, relu): stem conv2, transition1.1, fuse 1<-0,
# transition2 / fuse 2<-{0,1}, fuse 3<-1 chain, transition3 / fuse 3<-{0,1,2}
S2_PLANES = [(64, 64, 128, 96, True), (256, 64, 64, 48, True), (32, 64, 64, 48, False),
             (32, 128, 32, 24, False), (64, 128, 32, 24, True), (64, 64, 32, 24, True),
             (32, 256, 16, 12, False), (64, 256, 16, 12, False), (128, 256, 16, 12, True)]


def _bf(t):
    return t.to(torch.bfloat16).float()


@pytest.mark.parametrize("mode", ["s2conv", "generic"])
@pytest.mark.parametrize("cin,cout,h,w,relu", S2_PLANES)
def test_stride2_vs_reference(cin, cout, h, w, relu, mode, monkeypatch):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import hrnet
    monkeypatch.setenv("MVPOSE_NO_S2CONV", "1" if mode == "generic" else "0")
    spec, xi, yo, sd = hrnet.conv_spec(cin, cout, h, w, k=3, stride=2, relu=relu, seed=cin + cout)
    n = 7
    g = hrnet.ConvGraph(spec, xi, yo, max_batch=n)
    gen = torch.Generator().manual_seed(cin * 7 + h)
    x = torch.randn((n, h, w, cin), generator=gen).bfloat16()
    out = torch.empty((n, h // 2, w // 2, cout), dtype=torch.bfloat16, device="cuda")
    g.run(x.cuda(), out)
    torch.cuda.synchronize()
    g.close()
    wt, b = hrnet.fold_bn(sd, "c", "bn")
    wt = _bf(torch.from_numpy(np.ascontiguousarray(wt.transpose(0, 3, 1, 2))).float())
    z = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), wt, stride=2, padding=1)
    z = z + torch.from_numpy(b).float()[None, :, None, None]
    ref = _bf(torch.relu(z) if relu else z).permute(0, 2, 3, 1)
    got = out.float().cpu()
    rel = (torch.linalg.vector_norm(got - ref) / torch.linalg.vector_norm(ref)).item()
    mx = (got - ref).abs().max().item()
    print(f"{mode} {cin}->{cout} {h}x{w}/2 relu={relu}: rel L2 {rel:.2e}, max abs {mx:.3e}")
    assert rel <= 4e-3 and mx <= 3 * ref.abs().max().item() * 2.0 ** -8


@pytest.mark.parametrize("cin,cout,h,w", [(64, 64, 128, 96), (256, 64, 64, 48)])
def test_generic_stride2_tile_shapes_bit_identical(cin, cout, h, w, monkeypatch):
    """The generic kernel's tile shapes differ only in which workgroup computes a pixel
    (same K order and epilogue): the 8-wave 16x8 tiles deployed for the Cin >= 64 planes
    equal the 4-wave tiles (MVPOSE_S2_TILE=7) bit for bit, at a batch (7) whose last
    tile rows are partial in no dimension but whose crop count is odd."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import hrnet
    monkeypatch.setenv("MVPOSE_NO_S2CONV", "1")
    spec, xi, yo, _ = hrnet.conv_spec(cin, cout, h, w, k=3, stride=2, relu=True, seed=3)
    n = 7
    g = hrnet.ConvGraph(spec, xi, yo, max_batch=n)
    x = torch.randn((n, h, w, cin), generator=torch.Generator().manual_seed(5)).bfloat16().cuda()
    outs = []
    for v in ("0", "7", "1", "2"):
        monkeypatch.setenv("MVPOSE_S2_TILE", v)
        out = torch.full((n, h // 2, w // 2, cout), float("nan"), dtype=torch.bfloat16, device="cuda")
        g.run(x, out)
        torch.cuda.synchronize()
        outs.append(out.cpu())
    g.close()
    assert not torch.isnan(outs[0].float()).any()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
