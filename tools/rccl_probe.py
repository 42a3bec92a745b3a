import sys, os
sys.path.insert(0, os.getcwd())
import torch
from aios_amd.runtime import native
m = native.require()
print("available", m.RcclComm.available(), flush=True)
uid = m.RcclComm.unique_id(); print("uid", len(uid), flush=True)
c = m.RcclComm(0, 1, 0, uid); print("comm ok", c.rank, c.world, flush=True)
print("error?", flush=True); print(c.error(), flush=True)
d = torch.randn(1024, device="cuda"); r = torch.zeros(1024, device="cuda")
c.allreduce(d.data_ptr(), 1024, r.data_ptr(), torch.cuda.current_stream().cuda_stream); torch.cuda.synchronize()
print("allreduce ok", torch.allclose(r, d), flush=True)
