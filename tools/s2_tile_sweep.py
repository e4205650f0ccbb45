"""Tile-shape sweep for the generic conv_mfma_kernel on the two stride-2 planes that
stay on it (stem conv2 64@128x96, transition1.1 256@64x48): MVPOSE_S2_TILE=0..6,
time per conv (HIP events on torch's stream) and max |diff| vs the default tile.
    python tools/s2_tile_sweep.py [batch] [reps] [variants, e.g. 0,5]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"))
import torch  # noqa: E402

from mvpose import hrnet  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
VARIANTS = [int(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else list(range(7))
for cin, cout, h, w in [(64, 64, 128, 96), (256, 64, 64, 48), (32, 32, 64, 48), (64, 64, 32, 24), (32, 32, 32, 24)]:
    spec, xi, yo, _ = hrnet.conv_spec(cin, cout, h, w, k=3, stride=2, relu=True, seed=1)
    g = hrnet.ConvGraph(spec, xi, yo, max_batch=n)
    x = torch.randn((n, h, w, cin), device="cuda").bfloat16()
    ref = None
    for v in VARIANTS:
        os.environ["MVPOSE_S2_TILE"] = str(v)
        y = torch.empty((n, h // 2, w // 2, cout), device="cuda", dtype=torch.bfloat16)
        for _ in range(3):
            g.run(x, y)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            g.run(x, y)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        if ref is None:
            ref = y.float()
        d = (y.float() - ref).abs().max().item()
        flop = 2.0 * n * (h // 2) * (w // 2) * cout * cin * 9
        print(f"{cin:3d}->{cout:3d} {h:3d}x{w:<3d} tile{v}: {us:7.1f} us {flop / us / 1e6:6.1f} TFLOP/s "
              f"maxdiff {d:.3g}", flush=True)
    g.close()
