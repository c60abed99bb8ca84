"""Build-container only (imports /root/reference, like tests/golden/make_golden.py): time one
deterministic BYOL train step of the REFERENCE (src/models/byol.py + torch AdamW, the
train_byol.py:56-74 loop body) and of the oracle restatement on the same CPU, same threads,
same WavLM-Large weights and inputs (B=2 x 8 s), so bench.py's cpu_baseline (the oracle, timed
on the GPU box) can be related to the reference's own CPU speed. Prints one JSON line."""
import json
import os
import sys
import tempfile
import time

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import make_golden as MG  # noqa: E402
from nrse_amd import arch as A  # noqa: E402
from oracle import wavlm_byol as O  # noqa: E402

sys.path.insert(0, MG.REF)   # the reference's src/ ahead of the drop-in shim package's
threads = int(os.environ.get("THREADS", "8"))
torch.set_num_threads(threads)
B, L = 2, 128000
arch = A.LARGE.deterministic()
clean, noisy = MG.make_inputs(B, L)
with tempfile.TemporaryDirectory() as td:
    from src.models.byol import byol_loss
    model, layout, flat = MG.build_reference_model(arch, 1024, 2048, 0.997, td)
    model.train()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-5, weight_decay=1e-5)

    def ref_step():
        pred, tproj = model(clean, noisy)
        loss = byol_loss(pred, tproj)
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)
        opt.step()
        model._update_target_network()

    ref_step()
    t0 = time.perf_counter(); ref_step(); t_ref = time.perf_counter() - t0
    del model, opt
st = O.OracleState(layout, flat)
c2, n2 = clean.squeeze(1), noisy.squeeze(1)
O.train_step(st, c2, n2, lr=1e-5, weight_decay=1e-5, ema_decay=0.997, step_seed=0)
t0 = time.perf_counter()
O.train_step(st, c2, n2, lr=1e-5, weight_decay=1e-5, ema_decay=0.997, step_seed=1)
t_or = time.perf_counter() - t0
print(json.dumps({"workload": "WavLM-Large BYOL det train step, B=2 x 8 s, CPU", "threads": threads,
                  "reference_s_per_step": round(t_ref, 2), "oracle_s_per_step": round(t_or, 2),
                  "oracle_over_reference": round(t_or / t_ref, 3),
                  "reference_pairs_per_s": round(B / t_ref, 4), "oracle_pairs_per_s": round(B / t_or, 4)}))
