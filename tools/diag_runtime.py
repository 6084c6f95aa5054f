import sys, os
order = sys.argv[1]
sys.path[:0] = ['.', 'car-trailer-mpc_amd']
if order == 'torch_first':
    import torch
    print("torch avail", torch.cuda.is_available(), torch.cuda.device_count())
import ttmpc
from oracle import ttmpc_oracle as to
from ttmpc.scenarios import synthetic_batch
s = ttmpc.BatchSolver(20, to.DEFAULT_PARAMS, to.DEFAULT_Q, to.DEFAULT_R, to.MPC_XLB, to.MPC_XUB, to.MPC_ULB, to.MPC_UUB)
x0, xr, ur = synthetic_batch(16, 20, seed=1)
X, U, st, it, kk = s.solve(x0, xr, ur)
print(order, "solve ok", st.tolist())
import torch
print("torch avail", torch.cuda.is_available())
t = torch.zeros(4, device='cuda'); print(t.sum().item())
with open('/proc/self/maps') as f:
    libs = sorted({l.split()[-1] for l in f if 'amdhip' in l or 'hsa-runtime' in l})
print(libs)
