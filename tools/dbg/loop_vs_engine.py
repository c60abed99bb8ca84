import os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "noise-robust-speech-embedding_amd")]
from nrse_amd import arch as A, _lib
from nrse_amd.engine import ByolEngine
from src.models.byol import BYOLSpeechModel, byol_loss
_lib.init_device(0)
dtype = torch.bfloat16 if sys.argv[1] == "bf16" else torch.float32
arch = A.TINY.deterministic()
config = {"model": {"name": "nrse/wavlm-tiny", "projection_dim": 256, "prediction_dim": 512, "ema_decay": 0.99},
          "training": {"learning_rate": 1e-5, "weight_decay": 1e-5, "seed": 3}}
model = BYOLSpeechModel(config, compute_dtype=dtype, arch=arch)
flat0 = model.engine.online.detach().clone()
eng = ByolEngine(arch, 256, 512, compute_dtype=dtype, init_flat=flat0.cpu())
eng.cfg.ema_decay, eng.cfg.weight_decay = 0.99, 1e-5
opt = torch.optim.AdamW(model.parameters(), lr=1e-5, weight_decay=1e-5)
g = torch.Generator().manual_seed(1)
def rel(a, b): return float((a.double() - b.double()).norm() / b.double().norm())
for step in range(3):
    c = torch.randn(4, 16000, generator=g).cuda(); n = c + 0.3 * torch.randn(4, 16000, generator=g).cuda()
    model.train()
    p, t = model(c, n)
    loss = byol_loss(p, t)
    opt.zero_grad(); loss.backward()
    gl = model.online_flat.grad.clone()
    torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
    opt.step(); model._update_target_network()
    le = eng.train_step(c, n, lr=1e-5, step_seed=step)
    torch.cuda.synchronize()
    print(step, "loss", float(loss), float(le), "grad rel", rel(gl, eng.grad), "online rel-diff",
          float((model.engine.online - eng.online).abs().max()), "target", float((model.engine.target - eng.target).abs().max()),
          "shadow", None if dtype == torch.float32 else float((model.engine.online_sh.float() - eng.online_sh.float()).abs().max()),
          "tshadow", None if dtype == torch.float32 else float((model.engine.target_sh.float() - eng.target_sh.float()).abs().max()),
          "m", float((opt.state[model.online_flat]['exp_avg'] - eng.m).abs().max()))
