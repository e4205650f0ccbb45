"""Diagnostics: the fused dwpw ops of a small forward against the unfused graph (which channels /
pixels differ).  python tools/dwpw_diag.py [size] [n]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"), os.path.join(ROOT, "tests")]
from mvpose import rtmdet as D  # noqa: E402


def main(size=128, n=2):
    sd = D.random_state_dict(0)
    rng = np.random.default_rng(5)
    frames = torch.from_numpy(rng.integers(0, 256, (n, size * 9 // 8, 2 * size, 3), dtype=np.uint8)).cuda()
    dets = {}
    for fuse in ("0", "1"):
        os.environ["MVPOSE_DET_DWPW"] = fuse
        dets[fuse] = D.RTMDetector(sd, max_batch=n, size=size)
    s1, s0 = dets["1"].spec, dets["0"].spec
    for k, op in enumerate(s1.ops):
        if op.kind != D.DET_DWPW:
            continue
        name = s1.names[k].split("+")[-1]
        k0 = [i for i, nm in enumerate(s0.names) if nm == name][0]
        dets["1"].run_ops(frames, 0, k + 1)
        dets["0"].run_ops(frames, 0, k0 + 1)
        torch.cuda.synchronize()
        v, v0 = op.out, s0.ops[k0].out
        got = dets["1"].tensor(v.t, n).float().cpu()[..., v.coff:v.coff + v.c]
        ref = dets["0"].tensor(v0.t, n).float().cpu()[..., v0.coff:v0.coff + v0.c]
        bad = got != ref
        print(k, s1.names[k][:70], tuple(got.shape), "bad", int(bad.sum()), "of", bad.numel(), flush=True)
        if bad.any():
            idx = bad.nonzero()
            print("  frames", sorted(set(idx[:, 0].tolist()))[:8], "rows", sorted(set(idx[:, 1].tolist()))[:24])
            print("  cols", sorted(set(idx[:, 2].tolist()))[:24], "chans", sorted(set(idx[:, 3].tolist()))[:48])
            print("  sample got", got[tuple(idx[0].tolist())].item(), "ref", ref[tuple(idx[0].tolist())].item())
            break
    for d in dets.values():
        d.close()


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
