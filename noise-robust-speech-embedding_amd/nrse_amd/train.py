"""Training entry: the train_byol.py loop (train_byol.py:20-245) on the fused MI355X step.

    python -m nrse_amd.train --config <reference yaml> [--device cuda:0 --batch_size --epochs --lr]
    torchrun --nproc-per-node 8 -m nrse_amd.train --config ...      (data parallel, RCCL)

Per iteration (train_byol.py:47-77): H2D of raw waveforms -> fused SNR mix -> health checks
(device flags, no host sync) -> forward -> loss -> backward -> [grad all-reduce] -> clip(1.0) +
AdamW -> EMA -> cosine LR. Validation (evaluate_byol.py:68-123), EarlyStopping
(train_byol.py:82-116) and checkpoints in the reference's torch.save format
(train_byol.py:207-240, state-dict keys of BYOLSpeechModel) follow each epoch.
"""
from __future__ import annotations

import logging
import math
import os
import time

import torch

from . import ddp, params as PR
from .config import get_config
from .engine import compute_mode
from .data import create_dataloaders, seed_host_rng
from .health import HealthMonitor
from .model import BYOLSpeechModel

logger = logging.getLogger("nrse")


class EarlyStopping:
    """train_byol.py:82-116."""

    def __init__(self, patience=5, min_delta=0.0, mode="min"):
        self.patience, self.min_delta, self.mode = patience, min_delta, mode
        self.counter, self.best_score, self.early_stop = 0, None, False

    def __call__(self, score):
        if self.best_score is None:
            self.best_score = score
            return False
        improvement = (self.best_score - score > self.min_delta) if self.mode == "min" else \
            (score - self.best_score > self.min_delta)
        if improvement:
            self.best_score, self.counter = score, 0
        else:
            self.counter += 1
            if self.counter >= self.patience:
                self.early_stop = True
        return self.early_stop


class FusedAdamW(torch.optim.Optimizer):
    """AdamW over the flat online buffer, executed by the engine's fused clip+AdamW+EMA kernels;
    a torch Optimizer so torch's LR schedulers (CosineAnnealingLR) drive its lr."""

    def __init__(self, model: BYOLSpeechModel, lr: float, weight_decay: float):
        super().__init__([model.online_flat], dict(lr=lr, weight_decay=weight_decay))
        self.model = model

    @property
    def lr(self):
        return self.param_groups[0]["lr"]

    def _moments(self):
        e = self.model.engine
        e.sync_optimizer()
        return PR.named_views(e.layout, e.m), PR.named_views(e.layout, e.v)

    def state_dict(self):
        """torch.optim.AdamW.state_dict() layout (what train_byol.py:209-215 checkpoints): per
        online parameter tensor i, state[i] = {'step', 'exp_avg', 'exp_avg_sq'} (the engine's
        fused moments, reshaped to the parameter), one param group with AdamW's hyper-parameters.
        `param_groups[0]['param_names']` names each index with its state_dict key (the encoder's
        tensors are in the flat layout's order, not transformers' module order)."""
        e = self.model.engine
        mv, vv = self._moments()
        names = list(mv)
        state = {}
        if e.step_count > 0:
            step = torch.tensor(float(e.step_count))
            state = {i: {"step": step.clone(), "exp_avg": mv[k].detach().clone(),
                         "exp_avg_sq": vv[k].detach().clone()} for i, k in enumerate(names)}
        group = {k: v for k, v in self.param_groups[0].items() if k != "params"}
        group.update(betas=tuple(e.cfg.betas), eps=e.cfg.eps, amsgrad=False, maximize=False, foreach=None,
                     capturable=False, differentiable=False, fused=None,
                     params=list(range(len(names))), param_names=names)
        return {"state": state, "param_groups": [group]}

    def load_state_dict(self, state_dict):
        """Restore the moments, step count and lr / weight decay from `state_dict` in this
        class's format: each state index is matched to its tensor by `param_names`, and every
        moment must have exactly that tensor's shape. A plain AdamW state (no `param_names`) is
        refused: its index order is the owning module's parameter order, which the flat layout
        does not share, and moments of equal size would load into the wrong tensors silently."""
        e = self.model.engine
        mv, vv = self._moments()
        names = list(mv)
        group = state_dict["param_groups"][0]
        order = group.get("param_names")
        if not order:
            raise ValueError("optimizer state has no param_names: only states written by FusedAdamW.state_dict() "
                             "can be matched to the flat parameter layout")
        if len(order) != len(names) or set(order) != set(names):
            raise ValueError("optimizer state does not match this model's parameters")
        st = state_dict["state"]
        for i, k in enumerate(order):
            if i in st:
                for moment in ("exp_avg", "exp_avg_sq"):
                    if tuple(st[i][moment].shape) != tuple(mv[k].shape):
                        raise ValueError(f"optimizer state {moment} of {k}: shape {tuple(st[i][moment].shape)}, "
                                         f"expected {tuple(mv[k].shape)}")
        with torch.no_grad():
            if not st:
                e.m.zero_()
                e.v.zero_()
                e.step_count = 0
            for i, k in enumerate(order):
                if i in st:
                    mv[k].copy_(st[i]["exp_avg"])
                    vv[k].copy_(st[i]["exp_avg_sq"])
                    e.step_count = int(float(st[i]["step"]))
        for k in ("lr", "weight_decay", "initial_lr"):
            if k in group:
                self.param_groups[0][k] = group[k]

    def step(self, closure=None):  # used by the unfused path (autograd backward)
        eng = self.model.engine
        eng.sync_optimizer()
        eng.grad.copy_(self.model.online_flat.grad)
        eng.optimizer_step(self.lr)


def train_one_epoch(model, dataloader, optimizer, scheduler, device, config, allreduce=None, world=1, rank=0,
                    step0=0, max_steps=None, health=None):
    """train_byol.py:20-79 over the reference's dict batches -> (mean epoch loss, steps).
    The step is the engine's fused one; the health checks of :52-59 are read back `health.lag`
    steps late (nrse_amd/health.py), so no host sync happens inside the loop."""
    model.train()
    eng = model.engine
    # every step's loss lands in its own slot (train_step(loss_out=)): no per-step copy kernel
    try:
        n_slots = max(1, len(dataloader))
    except TypeError:           # a loader without a length
        n_slots = 1024
    losses = torch.empty(n_slots, device=eng.dev, dtype=torch.float32)
    steps = 0
    for batch in dataloader:
        if steps == losses.numel():   # more batches than the loader announced
            losses = torch.cat([losses, torch.empty_like(losses)])
        clean = batch["clean_input_values"].to(device, non_blocking=True)
        noisy = batch["noisy_input_values"].to(device, non_blocking=True)
        eng.train_step(clean.reshape(clean.shape[0], -1), noisy.reshape(noisy.shape[0], -1),
                       lr=optimizer.lr, step_seed=step0 + steps, rank=rank, allreduce=allreduce,
                       world_size=world, loss_out=losses[steps:steps + 1])
        if health is not None:
            health.record(step0 + steps, eng.health_buf, engine=eng)
        scheduler.step()
        steps += 1
        if max_steps is not None and step0 + steps >= max_steps:
            break
    if health is not None:
        health.flush()
    if not steps:
        return float("nan"), steps
    return float(losses[:steps].mean()), steps  # one host sync per epoch


@torch.no_grad()
def validate_model(model, val_loader, device, config, world=1):
    """evaluate_byol.py:68-123: per-SNR cosine similarity of online-encoder embeddings of the
    clean vs noisy views + validation BYOL loss, in eval mode. With world > 1 the sums are
    all-reduced, so every rank gets the same metrics (and the same early-stopping decision)."""
    model.eval()
    eng = model.engine
    snrs = list(config["data"]["snr_range"])
    sim_sum = torch.zeros(len(snrs), dtype=torch.float64, device=eng.dev)
    sim_cnt = torch.zeros(len(snrs), dtype=torch.float64, device=eng.dev)
    vl = torch.zeros(2, dtype=torch.float64, device=eng.dev)   # loss sum, batches
    for batch in val_loader or []:
        c = batch["clean_input_values"].to(device).reshape(batch["clean_input_values"].shape[0], -1)
        n = batch["noisy_input_values"].to(device).reshape(c.shape[0], -1)
        ec = eng.embed(c)
        en = eng.embed(n)
        s = torch.nn.functional.cosine_similarity(ec, en, dim=1).double()
        for k, snr in enumerate(snrs):
            m = (batch["snr"].to(eng.dev) == snr)
            sim_sum[k] += (s * m).sum()
            sim_cnt[k] += m.sum()
        _, _, loss = eng.eval_forward(c, n)
        vl[0] += loss.double().sum()
        vl[1] += 1
    if world > 1:
        for t in (sim_sum, sim_cnt, vl):
            ddp.all_reduce_sum(t)
    model.train()
    avg = {snr: (float(sim_sum[k] / sim_cnt[k]) if float(sim_cnt[k]) > 0 else 0.0) for k, snr in enumerate(snrs)}
    val_loss = float(vl[0] / vl[1]) if float(vl[1]) > 0 else float("inf")
    return val_loss, {"val_loss": val_loss, "val_avg_similarity": sum(avg.values()) / len(avg) if avg else 0.0,
                      "val_similarities": avg}


def main(argv=None):
    config = get_config(argv)
    rank, world, local = ddp.init_from_env()
    logging.basicConfig(level=getattr(logging, config.get("logging", {}).get("level", "INFO")))
    device = torch.device(config["device"]) if world == 1 else torch.device("cuda", local)
    torch.cuda.set_device(device)
    t = config["training"]
    torch.manual_seed(t.get("seed", 42))
    seed_host_rng(t.get("seed", 42), rank)
    os.makedirs(t["checkpoint_dir"], exist_ok=True)
    os.makedirs(t["log_dir"], exist_ok=True)
    dtype, wsplit = compute_mode(config["runtime"]["dtype"])
    model = BYOLSpeechModel(config, device=device, compute_dtype=dtype, weight_split=wsplit)
    train_loader, val_loader = create_dataloaders(config, device=device, rank=rank, world=world)
    optimizer = FusedAdamW(model, lr=float(t["learning_rate"]), weight_decay=float(t["weight_decay"]))
    total_steps = max(1, len(train_loader) * int(t["num_epochs"]))
    scheduler = torch.optim.lr_scheduler.CosineAnnealingLR(optimizer, T_max=total_steps)
    metric = t.get("early_stopping_metric", "val_loss")
    stopper = EarlyStopping(t.get("early_stopping_patience", 5), t.get("early_stopping_min_delta", 0.0),
                            "min" if metric == "val_loss" else "max")
    allreduce = ddp.GradAllReduce(wire_dtype=torch.bfloat16 if config["runtime"].get("bf16_allreduce") else None) \
        if world > 1 else None
    if world > 1 and config["runtime"].get("sync_bn"):
        model.engine.sync_bn = ddp.SyncBN()
    health = HealthMonitor()
    best_loss, best_sim, step = float("inf"), 0.0, 0
    max_steps = config["runtime"].get("max_steps")
    for epoch in range(int(t["num_epochs"])):
        t0 = time.perf_counter()
        ep_loss, n = train_one_epoch(model, train_loader, optimizer, scheduler, device, config, allreduce,
                                     world, rank, step, max_steps, health)
        step += n
        val_loss, vm = validate_model(model, val_loader, device, config, world)
        if rank == 0:
            print(f"Epoch {epoch + 1}/{t['num_epochs']} - Train Loss: {ep_loss:.4f}, Val Loss: {val_loss:.4f}, "
                  f"Val Avg Similarity: {vm['val_avg_similarity']:.4f} ({n} steps, "
                  f"{n * int(t['batch_size']) * world / (time.perf_counter() - t0):.1f} pairs/s)", flush=True)
        # early stopping first: on the stopping epoch the reference breaks before any save
        # (train_byol.py:192-196, then the checkpoints :207-240)
        if stopper(val_loss if metric == "val_loss" else vm["val_avg_similarity"]):
            if rank == 0:
                print(f"Early stopping triggered after epoch {epoch + 1}")
            break
        if rank == 0:
            ck = {"epoch": epoch, "model_state_dict": model.state_dict(), "optimizer_state_dict": optimizer.state_dict(),
                  "loss": val_loss, "similarity": vm["val_avg_similarity"]}
            if val_loss < best_loss:
                best_loss = val_loss
                torch.save(ck, os.path.join(t["checkpoint_dir"], "best_val_loss.pt"))
            if vm["val_avg_similarity"] > best_sim:
                best_sim = vm["val_avg_similarity"]
                torch.save(ck, os.path.join(t["checkpoint_dir"], "best_val_similarity.pt"))
            if epoch == int(t["num_epochs"]) - 1:
                torch.save(ck, os.path.join(t["checkpoint_dir"], "last_model.pt"))
        if max_steps is not None and step >= max_steps:
            break
    if world > 1:
        torch.distributed.destroy_process_group()
    if rank == 0:
        print("Training complete!")


if __name__ == "__main__":
    main()
