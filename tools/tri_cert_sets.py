import sys, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/multi-camera_3d_pose_estimation_amd')
from mvpose import synthetic as syn
from oracle import cv_ref
from mvpose import ops as _ops  # pack_camera only (no GPU use)
recs = []
def mk(kind, seed, T=20000, noise=1.0):
    cams = syn.make_rig(2, seed=seed)
    if kind == 'pose':
        k = syn.make_kpts_2d(syn.make_poses(T, seed=seed+1), cams, seed=seed+2, noise_px=noise)
    else:
        rng = np.random.default_rng(seed)
        k = np.zeros((T, 17, 3, 2), np.float32)
        k[:, :, 0] = rng.uniform(0, 1280, (T, 17, 2)); k[:, :, 1] = rng.uniform(0, 720, (T, 17, 2)); k[:, :, 2] = 1
    pts = np.ascontiguousarray(k[:, :, :2, :].reshape(-1, 2, 2).transpose(0, 2, 1)).astype(np.float32)  # (n, view, xy)
    cp = np.stack([_ops.pack_camera(c['K'], c['R'], c['T'], c['dist']) for c in cams])
    return pts, cp
sets = [('pose', 51, 1.0), ('pose', 52, 0.0), ('pose', 53, 40.0), ('pose', 71, 0.5), ('rand', 61, 0), ('pose', 5, 3.0), ('pose', 6, 1.0)]
with open('/tmp/tri/sets.bin', 'wb') as f:
    np.array([len(sets)], np.int64).tofile(f)
    for kind, seed, noise in sets:
        pts, cp = mk(kind, seed, T=20000 if kind == 'pose' else 5000, noise=noise)
        np.array([pts.shape[0]], np.int64).tofile(f); cp.astype(np.float64).tofile(f); pts.tofile(f)
print('ok')
