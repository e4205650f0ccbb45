"""Host-side cost of small host-to-device copies (pageable vs a reused pinned buffer)."""
import time
import numpy as np
import torch
a = np.arange(300, dtype=np.int32)
dev = "cuda:0"
torch.from_numpy(a).to(dev)
torch.cuda.synchronize()
pin = torch.empty(4096, dtype=torch.int32).pin_memory()
for _ in range(3):
    t = time.perf_counter(); torch.from_numpy(a).to(dev); t1 = time.perf_counter()
    pin[:a.size].copy_(torch.from_numpy(a)); x = pin[:a.size].to(dev, non_blocking=True); t2 = time.perf_counter()
    torch.zeros(10000, dtype=torch.int32, device=dev); t3 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"pageable {1e6*(t1-t):.1f} us, pinned async {1e6*(t2-t1):.1f} us, zeros {1e6*(t3-t2):.1f} us")
