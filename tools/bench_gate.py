import os, sys
sys.path.insert(0, os.path.join(os.getcwd(), "noise-robust-speech-embedding_amd"))
import torch
from nrse_amd import _lib, kernels as K
_lib.init_device(0)
B, T, H = 32, 399, 16
x1 = torch.randn(B * T, H * 64, device="cuda").to(torch.bfloat16)
W = torch.randn(8, 64, device="cuda") * 0.1; bv = torch.randn(8, device="cuda"); c = torch.randn(H, device="cuda")
dgate = torch.randn(B, H, T, device="cuda"); dx1 = torch.randn(B * T, H * 64, device="cuda")
dW = torch.zeros(8, 64, device="cuda"); db = torch.zeros(8, device="cuda"); dc = torch.zeros(H, device="cuda")
f = lambda: K.gate_bwd(x1, W, bv, c.view(1, H, 1, 1), dgate, dx1, dW, db, dc, B, T, H)
for _ in range(3): f()
torch.cuda.synchronize()
s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(20): f()
e.record(); torch.cuda.synchronize()
print(f"gate_bwd {s.elapsed_time(e) / 20 * 1e3:.1f} us")
