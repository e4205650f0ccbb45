"""tblock64 determinism under LDS pollution: the same block run repeatedly with other
LDS-heavy kernels in between (N = 2, 5, 7, 37)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"))
import torch  # noqa: E402

from mvpose import hrnet  # noqa: E402

spec, xi, yo, _ = hrnet.basic_block_spec(64, 32, 24, seed=13, n_blocks=2)
os.environ["MVPOSE_NO_TBLOCK64"] = "1"
gref = hrnet.ConvGraph(spec, xi, yo, max_batch=64)
os.environ["MVPOSE_NO_TBLOCK64"] = "0"
gf = hrnet.ConvGraph(spec, xi, yo, max_batch=64)
spec2, xi2, yo2, _ = hrnet.basic_block_spec(32, 64, 48, seed=3, n_blocks=1)
gp = hrnet.ConvGraph(spec2, xi2, yo2, max_batch=64)
junk = (torch.randn((64, 64, 48, 32), device="cuda") * 100).bfloat16()
junk_out = torch.empty_like(junk)
for n in (2, 5, 7, 37):
    x = torch.randn((n, 32, 24, 64), device="cuda").bfloat16()
    ref = torch.empty_like(x)
    gref.run(x, ref)
    bad = 0
    for it in range(20):
        gp.run(junk, junk_out)  # pollute LDS
        y = torch.full_like(x, float("nan"))
        gf.run(x, y)
        torch.cuda.synchronize()
        if not torch.equal(y, ref):
            bad += 1
            d = (y.float() - ref.float()).abs()
            idx = (d > 0).nonzero()
            print(f"n={n} it={it}: {int((d > 0).sum())} diffs, crops {sorted(set(idx[:, 0].tolist()))[:8]}, rows "
                  f"{sorted(set(idx[:, 1].tolist()))[:12]}, cols {sorted(set(idx[:, 2].tolist()))[:12]}, "
                  f"ch {sorted(set(idx[:, 3].tolist()))[:8]}", flush=True)
    print(f"n={n}: {bad}/20 runs differ", flush=True)
