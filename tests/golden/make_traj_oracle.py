"""Control fixture for tests/test_trajectory_gpu.py: the ORACLE's split-weight fp8 restatement
(oracle/wavlm_byol.py: bf16 activation operands at O.SPLIT_WEIGHT_SITES, the fp8 corrections at
O.SPLIT8_SITES, gradients rounded at the same sites) replaying the reference trajectory of
traj_large_3s.npz -- same weights, batches and lr schedule. It measures how far a bf16-precision
BACKWARD alone carries the trajectory from the f32 reference in this regime (random-init WavLM-Large,
BatchNorm heads over 4 near-identical embeddings), independent of the HIP kernels. Oracle output,
not reference output: runs anywhere the oracle runs (CPU, ~3 min at 8 threads).

Usage: PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_traj_oracle.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "noise-robust-speech-embedding_amd"))
sys.dont_write_bytecode = True

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import wavlm_byol as O  # noqa: E402
from nrse_amd import arch as A, params as PR  # noqa: E402


def make_inputs(B, L, seed):
    g = torch.Generator().manual_seed(seed)
    c = torch.randn(B, 1, L, generator=g)
    n = c + 0.3 * torch.randn(B, 1, L, generator=g)
    return c.squeeze(1), n.squeeze(1)


def rel(a, b):
    a, b = torch.as_tensor(a).double(), torch.as_tensor(b).double()
    return float((a - b).norm() / b.norm())


def main():
    torch.set_num_threads(8)
    z = np.load(os.path.join(HERE, "traj_large_3s.npz"))
    arch = A.LARGE.deterministic()
    layout = PR.byol_layout(arch, int(z["proj_dim"]), int(z["pred_dim"]))
    flat = PR.init_byol_flat(layout, int(z["seed"]))
    B, L, seed = int(z["B"]), int(z["L"]), int(z["seed"])
    P = O.split_flat(layout, flat)["encoder"]
    hc, hn = make_inputs(B, L, seed + 99)
    with torch.no_grad():
        e0 = O.encoder_forward(P, arch, hc, train=False).mean(1)
    motion = rel(e0, z["held_emb"])       # how far the reference's own held-out embedding moved
    names = [f"encoder.layers.{li}.{n}" for li in range(arch.layers)
             for n in ("attention.q_proj.weight", "attention.k_proj.weight", "attention.v_proj.weight",
                       "attention.out_proj.weight", "feed_forward.intermediate_dense.weight",
                       "feed_forward.output_dense.weight")]
    e8 = O.lo8_exponent([P[n] for n in names])
    st = O.OracleState(layout, flat)
    losses, norms = [], []
    O.set_operand_dtype(torch.bfloat16, O.SPLIT_WEIGHT_SITES)
    O.set_split8(O.SPLIT8_SITES, e8, O.conv_lo8_exponent(P, arch))
    try:
        for i in range(int(z["steps"])):
            c, n = make_inputs(B, L, seed + 100 + i)
            r = O.train_step(st, c, n, lr=float(z["lrs"][i]), weight_decay=float(z["wd"]), ema_decay=float(z["ema"]),
                             step_seed=i)
            losses.append(r["loss"])
            norms.append(r["grad_norm"])
            print(f"step {i}: loss {r['loss']:.6f} (ref {float(z['losses'][i]):.6f}) grad norm {r['grad_norm']:.4f} "
                  f"(ref {float(z['grad_norms'][i]):.4f})", flush=True)
    finally:
        O.set_operand_dtype(None)
        O.set_split8(None)
    with torch.no_grad():
        e = O.encoder_forward(O.split_flat(layout, st.online)["encoder"], arch, hc, train=False).mean(1)
        et = O.encoder_forward(O.split_flat(layout, st.target, target=True)["encoder"], arch, hn,
                               train=False).mean(1)
    res = dict(losses=np.array(losses), grad_norms=np.array(norms), held_emb=e.numpy(), held_temb=et.numpy(),
               held_emb_dev=rel(e, z["held_emb"]), held_temb_dev=rel(et, z["held_temb"]),
               ref_motion=motion)
    np.savez_compressed(os.path.join(HERE, "traj_large_3s_oracle_split8.npz"), **res)
    print(f"oracle split8 trajectory: held emb {res['held_emb_dev']:.3e} from the reference (its own motion "
          f"from init {motion:.3e}), target {res['held_temb_dev']:.3e}")


if __name__ == "__main__":
    main()
