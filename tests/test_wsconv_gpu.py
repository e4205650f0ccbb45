"""GPU parity of the branch-plane BasicBlock convolutions (csrc/wsconv.hip for
64 ch @ 32x24 and 128 ch @ 16x12; conv.hip / block.hip for the other planes)
against a torch fp32 restatement that rounds to bf16 at the same tensor
boundaries as the device graph (bf16 weights and activations, f32 bias and
accumulation).  The weight-stationary kernel sums K in (tap, cin) order and the
generic kernel in (cin chunk, tap) order, so both are compared against the
reference with a tolerance, not bit for bit:
  relative L2 error <= 4e-3, and |dev - ref| <= 3 bf16 ulps of max|ref|."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

PLANES = [(32, 64, 48), (64, 32, 24), (128, 16, 12), (256, 8, 6)]


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


def _run(c, h, w, n, n_blocks, seed, monkeypatch, ws):
    from mvpose import hrnet
    monkeypatch.setenv("MVPOSE_WSCONV64", "1")
    spec, xi, yo, sd = hrnet.basic_block_spec(c, h, w, seed=seed, n_blocks=n_blocks)
    if ws:
        monkeypatch.delenv("MVPOSE_NO_WSCONV", raising=False)
    else:
        monkeypatch.setenv("MVPOSE_NO_WSCONV", "1")
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
    for ws in (True, False):
        got, ref = _run(c, h, w, n, 2, 3, monkeypatch, ws)
        assert torch.isfinite(got).all()
        rel = (torch.linalg.vector_norm(got - ref) / torch.linalg.vector_norm(ref)).item()
        mx = (got - ref).abs().max().item()
        scale = ref.abs().max().item()
        print(f"C={c} {h}x{w} ws={ws}: rel L2 {rel:.2e}, max abs {mx:.3e} (max|ref| {scale:.2f})")
        assert rel <= 4e-3
        assert mx <= 3 * scale * 2.0 ** -8


@pytest.mark.parametrize("c,h,w", [(64, 32, 24), (128, 16, 12)])
def test_wsconv_batch_positions(c, h, w, monkeypatch):
    """A crop's output must not depend on its batch position or the batch size
    (tile scheduling over a persistent grid)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import hrnet
    monkeypatch.delenv("MVPOSE_NO_WSCONV", raising=False)
    monkeypatch.setenv("MVPOSE_WSCONV64", "1")
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
