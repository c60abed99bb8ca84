"""hipBLASLt (torch) rates on every GEMM of the WavLM-Large step, for reference against nrse_gemm:
forward y = x W^T, dgrad dx = dy W, wgrad dW = dy^T x (bf16 in; f32 out where torch allows)."""
import torch

dev = "cuda"
M = 12768


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


for name, N, Kd in (("qkv", 3072, 1024), ("out", 1024, 1024), ("ffn1", 4096, 1024), ("ffn2", 1024, 4096)):
    x = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
    w = torch.randn(N, Kd, device=dev).to(torch.bfloat16)
    dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
    fl = 2.0 * M * N * Kd
    r = {}
    r["fwd"] = timeit(lambda: torch.mm(x, w.t()))
    r["dgrad"] = timeit(lambda: torch.mm(dy, w))
    r["wgrad_bf16"] = timeit(lambda: torch.mm(dy.t(), x))
    try:
        r["wgrad_f32"] = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
    except Exception as ex:  # noqa
        r["wgrad_f32"] = float("nan")
    print(f"{name} {M}x{N}x{Kd}: " + " ".join(f"{k} {fl / v / 1e9:.0f}TF" for k, v in r.items()), flush=True)
