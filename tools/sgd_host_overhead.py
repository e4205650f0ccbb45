import os, sys, json, time
ROOT='/root/repo'
sys.path[:0]=[ROOT, ROOT+'/multi-camera_3d_pose_estimation_amd', ROOT+'/tests']
import numpy as np, torch
import bench
from mvpose import refine
from sgd_problem import BENCH_C5_KW, bench_c5_inputs
cams,g,x0=bench_c5_inputs(8,400)
lengths=json.load(open(ROOT+'/tests/golden/body_part_lengths.json'))['my_lengths']
camlist=[[c["K"], c["R"], c["T"], c["dist"]] for c in cams]
kw=dict(BENCH_C5_KW, body_lengths=dict(lengths), device='cuda:0')
G=torch.tensor(np.broadcast_to(g,(256,)+g.shape).copy(),device='cuda:0'); X=torch.tensor(np.broadcast_to(x0,(256,)+x0.shape).copy(),device='cuda:0')
refine.refine_trajectories(G,X,camlist,**kw); torch.cuda.synchronize()
orig=refine.call
stamps={}
def tc(name,*a):
    t=time.perf_counter(); r=orig(name,*a); stamps[name]=(t, time.perf_counter()); return r
refine.call=tc
for _ in range(3):
    torch.cuda.synchronize()
    t0=time.perf_counter(); refine.refine_trajectories(G,X,camlist,**kw); t1=time.perf_counter()
    torch.cuda.synchronize()
    s=stamps['mvp_sgd_refine']; w=stamps['mvp_sgd_workspace_floats']
    print(json.dumps({"host_total_us":(t1-t0)*1e6, "until_ws_call_us":(w[0]-t0)*1e6, "until_launch_us":(s[0]-t0)*1e6, "launch_call_us":(s[1]-s[0])*1e6}))
