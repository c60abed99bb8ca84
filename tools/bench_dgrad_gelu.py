"""The FFN-down dgrad of the step (dx[12768, 4096] = dy[12768, 1024] W2[1024, 4096], bf16 out) with
its epilogue variants, isolated, median of 5 rounds: plain, + GELU' from the bf16 pre-activation,
+ GELU' + the FFN-up bias column sums (the step's form), and the forward FFN-up of the same output
shape (TT, + bias + GELU + pre-activation) for comparison."""
import os, sys, statistics
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "noise-robust-speech-embedding_amd"))
import torch
from nrse_amd import kernels as K, _lib

_lib.init_device(0)
dev = "cuda"
M, H, F = 12768, 1024, 4096
dy = torch.randn(M, H, device=dev).to(torch.bfloat16)
w2 = (torch.randn(H, F, device=dev) * 0.03).to(torch.bfloat16)
pre = torch.randn(M, F, device=dev).to(torch.bfloat16)
dx = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
cs = torch.zeros(F, device=dev)
x = torch.randn(M, H, device=dev).to(torch.bfloat16)
w1 = (torch.randn(F, H, device=dev) * 0.03).to(torch.bfloat16)
b1 = torch.randn(F, device=dev)


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


forms = {
    "dgrad plain": lambda: K.linear_dgrad(dy, w2, dx),
    "dgrad +gelu'": lambda: K.linear_dgrad(dy, w2, dx, flags=_lib.EPI_GELU_BWD, aux=pre, ldaux=F),
    "dgrad +gelu' +colsum": lambda: K.linear_dgrad(dy, w2, dx, flags=_lib.EPI_GELU_BWD, aux=pre, ldaux=F, colsum=cs),
    "fwd ffn-up +gelu +aux": lambda: K.linear_fwd(x, w1, dx, bias=b1, flags=_lib.EPI_GELU, aux=pre, ldaux=F),
}
res = {k: [] for k in forms}
for _ in range(5):
    for k, f in forms.items():
        res[k].append(timeit(f))
fl = 2.0 * M * H * F
print("  ".join(f"{k} {statistics.median(v):.1f}us ({fl / statistics.median(v) / 1e6:.0f}TF)" for k, v in res.items()))
