"""Per-conv timing of HRNet-W32's 3x3/stride-2 convs at the bench batch:
s2conv.hip vs the generic conv_mfma_kernel (MVPOSE_NO_S2CONV=1).  HIP events on
torch's stream.   python tools/s2_bench.py [batch] [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"))
import torch  # noqa: E402

from mvpose import hrnet  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
# (cin, cout, h, w, calls per forward)
PLANES = [(64, 64, 128, 96, 1), (256, 64, 64, 48, 1), (32, 64, 64, 48, 7), (32, 32, 64, 48, 8),
          (32, 128, 32, 24, 6), (64, 128, 32, 24, 7), (64, 64, 32, 24, 2), (32, 32, 32, 24, 2),
          (32, 256, 16, 12, 2), (64, 256, 16, 12, 2), (128, 256, 16, 12, 3)]
tot = {"s2conv": 0.0, "generic": 0.0}
for cin, cout, h, w, calls in PLANES:
    for mode in ("generic", "s2conv"):
        os.environ["MVPOSE_NO_S2CONV"] = "1" if mode == "generic" else "0"
        spec, xi, yo, _ = hrnet.conv_spec(cin, cout, h, w, k=3, stride=2, relu=True, seed=1)
        g = hrnet.ConvGraph(spec, xi, yo, max_batch=n)
        x = torch.randn((n, h, w, cin), device="cuda").bfloat16()
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
        flop = 2.0 * n * (h // 2) * (w // 2) * cout * cin * 9
        byt = 2.0 * n * (h * w * cin + (h // 2) * (w // 2) * cout)
        tot[mode] += us * calls
        print(f"{cin:3d}->{cout:3d} {h:3d}x{w:<3d} x{calls} {mode:8s}: {us:7.1f} us  "
              f"{flop / us / 1e6:6.1f} TFLOP/s  {byt / us / 1e3:6.0f} GB/s", flush=True)
        g.close()
print(f"per forward: generic {tot['generic']:.0f} us, s2conv {tot['s2conv']:.0f} us")
