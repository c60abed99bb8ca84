"""AdamW + target EMA over one encoder layer's segment (12.6 M f32 weights, bf16 shadows), as
two passes (nrse_adamw, nrse_ema) and as one (nrse_adamw_params.ema_t); algorithmic bytes per
weight: 30 + 14 (two passes), 40 (fused), 44 (fused + zero_grad, the engine's form)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "noise-robust-speech-embedding_amd"))
import torch
from nrse_amd import kernels as K, _lib

_lib.init_device(0)
dev = "cuda"
n = int(os.environ.get("N", 12_596_224))
p, g, m, v, t = (torch.randn(n, device=dev) for _ in range(5))
sh = torch.empty(n, device=dev, dtype=torch.bfloat16); tsh = torch.empty_like(sh)
ss = torch.ones(1, device=dev, dtype=torch.float64)
kw = dict(lr=1e-4, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-2, step=5, max_norm=1.0, sumsq_buf=ss)


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


for _ in range(2):
    ta = timeit(lambda: K.adamw(p, g, m, v, sh, **kw))
    te = timeit(lambda: K.ema(t, p, tsh, 0.997))
    tf = timeit(lambda: K.adamw(p, g, m, v, sh, ema_t=t, ema_shadow=tsh, ema_decay=0.997, **kw))
    print(f"n={n}: adamw {ta:.1f}us ({30 * n / ta / 1e6:.2f} TB/s) + ema {te:.1f}us ({14 * n / te / 1e6:.2f} TB/s) = "
          f"{ta + te:.1f}us | fused {tf:.1f}us ({40 * n / tf / 1e6:.2f} TB/s)", flush=True)
    tz = timeit(lambda: K.adamw(p, g, m, v, sh, ema_t=t, ema_shadow=tsh, ema_decay=0.997, zero_grad=True, **kw))
    print(f"n={n}: fused + zero_grad {tz:.1f}us ({44 * n / tz / 1e6:.2f} TB/s)", flush=True)
