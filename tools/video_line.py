"""Print bench.py's video_decode line (host decoder at 1 / 16 threads, split decode onto the GPU)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"))
import bench
print(json.dumps(bench.video_decode_line(), indent=1))
