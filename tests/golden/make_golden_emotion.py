"""Golden fixture for the emotion head (BASELINE configs[3]) from the REFERENCE module itself.

Runs only in the build container: imports /root/reference src.models.emotion.EmotionClassifier
(and its AttentiveStatisticsPooling) with a stub encoder that returns a fixed hidden state, the
reference ccc_loss (src/train/dimentional_emotions.py:427-450 is restated, since importing that
module pulls wandb), and records the dimensional output, loss and head gradients with dropout off
(model.eval()). The GPU box only reads tests/golden/emotion_head.npz.

Usage: PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_emotion.py
"""
from __future__ import annotations

import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, "/root/reference")

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from src.models.emotion import EmotionClassifier
    torch.manual_seed(0)
    B, T, C, Hd = 5, 37, 256, 256
    L = 320 * (T - 1) + 400                     # samples whose WavLM frame count is T
    hidden = torch.randn(B, T, C) * 0.7

    class Stub(torch.nn.Module):
        output_dim = C

        def forward(self, x, attention_mask=None):
            return hidden

    model = EmotionClassifier(Stub(), hidden_dim=Hd, dropout=0.3, num_emotions=8)
    g = torch.Generator().manual_seed(3)
    with torch.no_grad():
        for n, p in model.named_parameters():
            p.copy_(torch.randn(p.shape, generator=g) * (0.05 if p.dim() > 1 else 0.1) +
                     (1.0 if n.endswith("1.weight") else 0.0))
    model.eval()                                 # dropout off
    mask = torch.ones(B, L)
    for b, keep in enumerate([L, L - 3000, L // 2, 4001, L]):
        mask[b, keep:] = 0
    labels = torch.rand(B, 3, generator=g) * 6 + 1
    x = torch.zeros(B, L)
    _, dim = model(x, attention_mask=mask, task="dimensional")
    loss = 0.0
    for i in range(3):                           # ccc_loss, dimentional_emotions.py:427-450
        p, t = dim[:, i], labels[:, i]
        mp, mt = p.mean(), t.mean()
        vp, vt = p.var(unbiased=False), t.var(unbiased=False)
        cov = ((p - mp) * (t - mt)).mean()
        loss = loss + 1 - 2 * cov / (vp + vt + (mp - mt) ** 2 + 1e-10)
    loss = loss / 3
    loss.backward()
    out = {"hidden": hidden.numpy(), "mask": mask.numpy(), "labels": labels.numpy(), "dim": dim.detach().numpy(),
           "loss": np.float64(float(loss))}
    from src.models.pool import AttentiveStatisticsPooling  # noqa: F401  (same module the model used)
    out["feat_lens"] = np.array(model.pooling.compute_length_from_mask(mask), dtype=np.int32)
    for n, p in model.named_parameters():
        out["param/" + n] = p.detach().numpy()
        if p.grad is not None:
            out["grad/" + n] = p.grad.numpy()
    np.savez_compressed(os.path.join(HERE, "emotion_head.npz"), **out)
    print("wrote emotion_head.npz", float(loss), out["feat_lens"])


if __name__ == "__main__":
    main()
