"""Which bf16 rounding sites carry the bf16 mode's embedding deviation from the reference?

Runs the oracle's eval forward of the online encoder at WavLM-Large on the byol_large fixture's
inputs (B = 4, 8 s; tests/golden/make_golden.py) with bf16 rounding on one site at a time (and on
all sites but one), and prints each embedding's rel-L2 against the reference's eval_emb.
CPU only (oracle = test infrastructure); results are quoted in DESIGN.md §6.

Usage: python tools/ablate_bf16_sites.py [--fixture byol_large.npz] [--threads 8]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "noise-robust-speech-embedding_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from nrse_amd import arch as A, params as PR  # noqa: E402
from oracle import wavlm_byol as O  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fixture", default="byol_large.npz")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--sets", default="single,leave_one,all")
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    z = np.load(os.path.join(ROOT, "tests", "golden", args.fixture))
    arch = A.LARGE.deterministic()
    layout = PR.byol_layout(arch, int(z["proj_dim"]), int(z["pred_dim"]))
    flat = PR.init_byol_flat(layout, int(z["seed"]))
    g = torch.Generator().manual_seed(int(z["seed"]) + 1)
    B, L = int(z["B"]), int(z["L"])
    clean = torch.randn(B, 1, L, generator=g).squeeze(1)
    P = O.split_flat(layout, flat)["encoder"]
    ref = torch.from_numpy(z["eval_emb"]).double()

    def run(sites, dtype=torch.bfloat16):
        O.set_operand_dtype(dtype, sites)
        try:
            with torch.no_grad():
                t0 = time.time()
                h = O.encoder_forward(P, arch, clean, train=False)
                emb = h.mean(1).double()
        finally:
            O.set_operand_dtype(None)
        return float((emb - ref).norm() / ref.norm()), time.time() - t0

    out = {}
    e, dt = run(None, torch.float32)
    out["none"] = e
    print(f"f32 (no rounding): {e:.3e}  ({dt:.1f} s)", flush=True)
    kinds = args.sets.split(",")
    if "all" in kinds:
        e, _ = run(None)
        out["all"] = e
        print(f"all sites: {e:.3e}", flush=True)
    if "single" in kinds:
        for s in O.SITES:
            e, _ = run([s])
            out["only_" + s] = e
            print(f"only {s:9s}: {e:.3e}", flush=True)
    if "leave_one" in kinds:
        for s in O.SITES:
            e, _ = run([x for x in O.SITES if x != s])
            out["all_but_" + s] = e
            print(f"all but {s:9s}: {e:.3e}", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
