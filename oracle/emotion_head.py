"""ORACLE (test infrastructure only — imported by tests/ and tests/golden/make_golden_emotion.py;
never by the product path).

fp32 PyTorch-eager CPU restatement of the dimensional-emotion head over a frozen encoder
(BASELINE configs[3]), written from the reference's algorithm:
  EmotionClassifier.forward    src/models/emotion.py:63-96 (task='dimensional')
  AttentiveStatisticsPooling   src/models/pool.py:11-19 (lengths from the sample mask), 25-58
  ccc_loss                     src/train/dimentional_emotions.py:427-450
  train step                   src/train/dimentional_emotions.py:306-338 (zero_grad, backward,
                               clip_grad_norm_(1.0), AdamW step)
Pinned against tests/golden/emotion_head.npz (the reference module itself on the same inputs,
dropout off) by tests/test_oracle_golden.py.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

# head parameter names in EmotionClassifier's state_dict order (encoder excluded)
def head_specs(C: int, hidden: int, num_emotions: int = 8):
    return [("pooling.sap_linear.weight", (C, C)), ("pooling.sap_linear.bias", (C,)), ("pooling.attention", (C, 1)),
            ("shared_fc.0.weight", (hidden, 2 * C)), ("shared_fc.0.bias", (hidden,)),
            ("shared_fc.1.weight", (hidden,)), ("shared_fc.1.bias", (hidden,)),
            ("categorical_fc.0.weight", (hidden, hidden)), ("categorical_fc.0.bias", (hidden,)),
            ("categorical_fc.1.weight", (hidden,)), ("categorical_fc.1.bias", (hidden,)),
            ("categorical_out.weight", (num_emotions, hidden)), ("categorical_out.bias", (num_emotions,)),
            ("dimensional_fc.0.weight", (hidden, hidden)), ("dimensional_fc.0.bias", (hidden,)),
            ("dimensional_fc.1.weight", (hidden,)), ("dimensional_fc.1.bias", (hidden,)),
            ("dimensional_out.weight", (3, hidden)), ("dimensional_out.bias", (3,))]


def feat_lengths(mask: torch.Tensor) -> list:
    """pool.py:11-19: frames from a (batch, samples) mask at a 20 ms hop."""
    wav_lens = mask.sum(dim=1)
    return (torch.div(wav_lens - 1, 16000 * 0.02, rounding_mode="floor") + 1).int().tolist()


def asp(xs: torch.Tensor, lens: list, P: dict) -> torch.Tensor:
    """pool.py:36-58."""
    out = []
    for x, n in zip(xs, lens):
        x = x[:n].unsqueeze(0)
        h = torch.tanh(F.linear(x, P["pooling.sap_linear.weight"], P["pooling.sap_linear.bias"]))
        w = torch.matmul(h, P["pooling.attention"]).squeeze(dim=2)
        w = F.softmax(w, dim=1).view(x.size(0), x.size(1), 1)
        mu = torch.sum(x * w, dim=1)
        rh = torch.sqrt((torch.sum((x ** 2) * w, dim=1) - mu ** 2).clamp(min=1e-5))
        out.append(torch.cat((mu, rh), 1).squeeze(0))
    return torch.stack(out)


def block(x, P, name, p_drop, train, drop_masks=None, key=None):
    """Linear -> LayerNorm -> ReLU -> Dropout (emotion.py:34-58)."""
    y = F.linear(x, P[name + ".0.weight"], P[name + ".0.bias"])
    y = F.layer_norm(y, (y.shape[-1],), P[name + ".1.weight"], P[name + ".1.bias"], 1e-5)
    y = F.relu(y)
    if train and p_drop > 0:
        y = y * drop_masks[key] / (1 - p_drop)
    return y


def dimensional_forward(hidden: torch.Tensor, lens: list, P: dict, p_drop=0.0, train=False, drop_masks=None):
    pooled = asp(hidden, lens, P)
    s = block(pooled, P, "shared_fc", p_drop, train, drop_masks, "shared")
    d = block(s, P, "dimensional_fc", p_drop, train, drop_masks, "dim")
    return F.linear(d, P["dimensional_out.weight"], P["dimensional_out.bias"]), pooled


def ccc_loss(pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """dimentional_emotions.py:427-450."""
    loss = pred.new_zeros(())
    if pred.size(0) > 1:
        for i in range(pred.size(1)):
            p, t = pred[:, i], target[:, i]
            mp, mt = torch.mean(p), torch.mean(t)
            vp, vt = torch.var(p, unbiased=False), torch.var(t, unbiased=False)
            cov = torch.mean((p - mp) * (t - mt))
            loss = loss + 1 - 2 * cov / (vp + vt + (mp - mt) ** 2 + 1e-10)
    return loss / pred.size(1)


def train_step(hidden, lens, labels, P: dict, lr: float, weight_decay: float, state: dict | None = None,
               p_drop=0.0, drop_masks=None):
    """One head step over a frozen encoder's output: returns (loss, grads, new params, state)."""
    Pv = {k: v.detach().clone().requires_grad_(True) for k, v in P.items()}
    out, _ = dimensional_forward(hidden, lens, Pv, p_drop, p_drop > 0, drop_masks)
    loss = ccc_loss(out, labels)
    loss.backward()
    # dimensional task: the categorical branch gets no gradient (torch leaves .grad None;
    # AdamW skips those parameters)
    names = [k for k in Pv if Pv[k].grad is not None]
    grads = {k: Pv[k].grad.detach().clone() for k in names}
    norm = math.sqrt(sum(float(g.double().pow(2).sum()) for g in grads.values()))
    coef = min(1.0, 1.0 / (norm + 1e-6))
    state = state if state is not None else {"step": 0, "m": {}, "v": {}}
    state["step"] += 1
    t = state["step"]
    b1, b2, eps = 0.9, 0.999, 1e-8
    newP = {k: v.detach().clone() for k, v in P.items()}
    for k in names:
        g = grads[k] * coef
        m = state["m"].get(k, torch.zeros_like(g)) * b1 + (1 - b1) * g
        v = state["v"].get(k, torch.zeros_like(g)) * b2 + (1 - b2) * g * g
        state["m"][k], state["v"][k] = m, v
        p = newP[k] * (1 - lr * weight_decay)
        mh = m / (1 - b1 ** t)
        vh = v / (1 - b2 ** t)
        newP[k] = p - lr * mh / (vh.sqrt() + eps)
    return float(loss), grads, newP, state, norm
