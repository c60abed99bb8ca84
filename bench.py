"""bench.py — BYOL utterance-pairs/sec for WavLM-Large, 8 s @ 16 kHz, batch 32 per GPU
(BASELINE.json metric), on N MI355X (one process per GPU, RCCL over xGMI).

A step = fused on-GPU SNR mix of 32 synthetic (clean, noise) pairs resident in HBM ->
BYOLSpeechModel forward (online on clean, target on noisy) -> BYOL loss -> backward ->
gradient all-reduce (N > 1) -> clip + AdamW -> target EMA, i.e. the train_one_epoch body
(train_byol.py:47-77) with the dataset mixing of src/data/augment.py moved on device.
Synthetic data, random-init WavLM-Large weights (pretrained weights are unavailable offline).

Usage: python bench.py [--gpus N --steps K --warmup W]; N > 1 under torch.distributed.run.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "noise-robust-speech-embedding_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
BF16_DENSE_PEAK_TFS = 2500.0   # dense bf16 MFMA (no sparsity)
F32_MFMA_PEAK_TFS = 157.3
SNR_RANGE = [2, 5, 10, 15, 20]  # config/default_wavlm-large_byol.yaml:28


def flops_per_pair(arch, L, executed):
    """Algorithmic FLOPs per BYOL pair (SURVEY §8d model): online fwd + 2x bwd + target fwd,
    conv0 input-grad excluded; `executed` = transformer layers run (online, target)."""
    conv = 0.0
    T = L
    cin = 1
    for k, s, c in zip(arch.conv_kernel, arch.conv_stride, arch.conv_dim):
        T = (T - k) // s + 1
        conv += 2.0 * T * c * cin * k
        cin = c
    H, Fd = arch.hidden, arch.ffn
    proj = 2.0 * T * cin * H
    pos = 2.0 * T * H * (H // arch.pos_groups) * arch.pos_kernel
    layer = 2.0 * T * H * 3 * H + 2.0 * T * H * H + 2 * 2.0 * T * T * H + 2 * 2.0 * T * H * Fd
    enc_fixed = conv + proj + pos
    online = enc_fixed + executed[0] * layer
    target = enc_fixed + executed[1] * layer
    return 3.0 * online + target, dict(conv=conv, proj=proj, pos=pos, layer=layer, T=T)


def cpu_baseline(arch_large, seconds_hint=20.0):
    """Oracle (fp32 PyTorch-eager CPU restatement, oracle/wavlm_byol.py) training step on the
    host cores: bounded sample of the same workload (B=2 pairs of 8 s, one timed step after one
    warm-up step). Reported baseline only."""
    from oracle import wavlm_byol as O
    from nrse_amd import params as PR
    # the GPU box's CPU share is 16 cores per GPU (os.cpu_count() reports the whole machine);
    # more threads oversubscribe and run slower
    torch.set_num_threads(max(1, min(os.cpu_count() or 1, 16)))
    layout = PR.byol_layout(arch_large, 1024, 2048)
    flat = PR.init_byol_flat(layout, 1234)
    st = O.OracleState(layout, flat)
    g = torch.Generator().manual_seed(0)
    B, L = 2, 128000
    clean = torch.randn(B, L, generator=g) * 0.1
    noisy = clean + 0.05 * torch.randn(B, L, generator=g)
    O.train_step(st, clean, noisy, lr=1e-5, weight_decay=1e-5, ema_decay=0.997, step_seed=0)
    t0 = time.perf_counter()
    O.train_step(st, clean, noisy, lr=1e-5, weight_decay=1e-5, ema_decay=0.997, step_seed=1)
    dt = time.perf_counter() - t0
    return {"value": B / dt, "unit": "pairs/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"oracle fp32 CPU train step, WavLM-Large, B={B} x 8 s, 1 warm-up + 1 timed step "
                      f"({dt:.1f} s/step), cpu={platform.processor() or platform.machine()}, "
                      f"os.cpu_count()={os.cpu_count()}"}


TRAFFIC_FILE = "r06_gemm_traffic.json"
SQ_TABLE_FILE = "r06_pmc_sq_table.json"


def gemm_traffic():
    """HBM bytes per nrse_gemm launch from the committed rocprofv3 PMC summary of the current
    step (tools/pmc_gemm.sh -> profiles/r06_gemm_traffic.json: FETCH_SIZE x 2 (gfx950
    correction) + WRITE_SIZE, averaged over the GEMM launches of a bench step). None if absent."""
    path = os.path.join(ROOT, "profiles", TRAFFIC_FILE)
    try:
        with open(path) as fh:
            return float(json.load(fh)["family_hbm_bytes_per_launch"])
    except (OSError, KeyError, ValueError):
        return None


def gemm_mfma_busy():
    """Matrix-pipe busy fraction of the 256x256 GEMM kernels from the committed counter pass
    (tools/pmc_sq.sh -> profiles/r06_pmc_sq_table.json): SQ_VALU_MFMA_BUSY_CYCLES over all
    SIMD-cycles of the launch (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs x 4 SIMDs), per step shape,
    isolated launches. None if absent."""
    path = os.path.join(ROOT, "profiles", SQ_TABLE_FILE)
    try:
        with open(path) as fh:
            t = json.load(fh)
        out = {}
        for k, v in t.items():
            if k.startswith("gemm256_kernel") and "mfma_busy" in v:
                name, grid, _ = k.rsplit(" ", 2)
                out[f"{name} ({int(grid) // 512} workgroups)"] = round(v["mfma_busy"], 3)
        return out
    except (OSError, KeyError, ValueError, IndexError):
        return None


def north_star_parity():
    """Embedding / prediction rel-L2 of the bf16sw mode against the reference's own outputs at 3 / 8 /
    12 s (tests/test_large_gpu.py::test_large_bf16sw_matches_reference records, committed under
    profiles/): the newest round's files."""
    out = {}
    for tag in ("3s", "8s", "12s"):
        for rnd in ("r06", "r05", "r04"):
            path = os.path.join(ROOT, "profiles", f"{rnd}_large_parity_bf16sw_{tag}.json")
            try:
                with open(path) as fh:
                    m = json.load(fh)
            except (OSError, ValueError):
                continue
            out[tag] = {"eval_emb_rel_l2": m.get("eval_emb"), "eval_pred_rel_l2": m.get("eval_pred"),
                        "eval_tproj_rel_l2": m.get("eval_tproj"), "source": f"profiles/{os.path.basename(path)}"}
            break
    out["bound"] = 1e-3
    return out


def bench_emotion(args):
    """configs[3]: one dimensional-emotion fine-tune iteration over the frozen WavLM-Large encoder
    (default_wavlm-large_emotion_dim_ft.yaml: batch 36, 5 s, hidden 1024, dropout 0.3, AdamW
    lr 1e-5 / wd 1e-4): encoder forward in train mode (no tape), head forward, CCC loss, head
    backward, clip + AdamW. Synthetic audio and A/V/D labels; 1 GPU."""
    from nrse_amd import arch as A, kernels as K
    from nrse_amd.emotion import EmotionDimTrainer, EmotionHead
    from nrse_amd.engine import ByolEngine
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    B = 36 if args.batch == 32 else args.batch
    L = int(5.0 * 16000)
    from nrse_amd.engine import compute_mode
    cdt, wsplit = compute_mode(args.dtype)
    eng = ByolEngine(A.LARGE, 1024, 2048, device=dev, compute_dtype=cdt, seed=1234, weight_split=wsplit)
    head = EmotionHead(1024, 1024, 8, dropout=0.3, device=dev, compute_dtype=cdt, seed=42)
    tr = EmotionDimTrainer(eng, head, lr=1e-5, weight_decay=1e-4)
    gen = torch.Generator(device=dev)
    gen.manual_seed(99)
    wav = torch.randn(B, L, device=dev, generator=gen) * 0.1
    labels = torch.rand(B, 3, device=dev, generator=gen) * 6 + 1
    lengths = torch.full((B,), L, dtype=torch.int64)
    for i in range(args.warmup):
        tr.train_step(wav, labels, lengths, step_seed=i)
    torch.cuda.synchronize()
    probe = []
    t0 = time.perf_counter()
    K.set_gemm_probe(probe)
    for i in range(args.steps):
        tr.train_step(wav, labels, lengths, step_seed=args.warmup + i)
    K.set_gemm_probe(None)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    gflops = sum(f for f, _, _, _ in probe)
    gms = sum(e0.elapsed_time(e1) for _, e0, e1, _ in probe)
    tfs = gflops / (gms * 1e-3) / 1e12 if gms > 0 else 0.0
    result = {"metric": "emotion-dim fine-tune utterances/sec, frozen WavLM-large encoder, 5s@16kHz, batch=36",
              "value": round(B * args.steps / dt, 3), "unit": "utterances/s", "n_gpus": 1, "steps": args.steps,
              "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 2), "higher_is_better": True,
              "scaling": "none", "vs_baseline": None, "dtype": args.dtype,
              "data": "synthetic 5 s audio and A/V/D labels, random-init encoder and head",
              "config": {"workload": "configs[3]: dimensional emotion head (attentive statistics pooling, shared + "
                                     "dimensional FC, CCC loss) over the frozen encoder", "global_batch": B,
                         "seq_len": L, "frames": A.LARGE.frames(L)},
              "roofline": {"bound": "mfma", "kernel": "nrse_gemm (all launches in the timed region)",
                           "achieved": round(tfs, 1), "peak": BF16_DENSE_PEAK_TFS, "unit": "TFLOP/s",
                           "frac": round(tfs / BF16_DENSE_PEAK_TFS, 4), "launches": len(probe)},
              "loss_last": round(float(head.loss_buf), 5)}
    print(json.dumps(result), flush=True)


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`--gpus N > 1` without a torch.distributed environment: start the N rank processes here
    (one per GPU, torch.distributed.run on 127.0.0.1) as children, before this process has made
    any GPU call, and return their exit status. Each rank re-runs this script with the same
    arguments and finds WORLD_SIZE set."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver (RCCL)
    env.setdefault("OMP_NUM_THREADS", "4")
    import subprocess
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "bf16sw", "f32"],
                    help="bf16 (the metric's mode), bf16sw (bf16 activations x split hi+lo bf16 weights in the "
                         "forward: embeddings within the north-star 1e-3), f32 (exact parity mode)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-north-star", action="store_true",
                    help="skip the north-star mode's (bf16sw) second timed run after the bf16 one (N = 1, fixed)")
    ap.add_argument("--detail", default=None, help="write per-shape GEMM timings here (json)")
    ap.add_argument("--serial-optimizer", action="store_true",
                    help="clip/AdamW/EMA on the main stream after backward (default: overlapped per layer "
                         "with the next step's forward, as the training loop runs it)")
    ap.add_argument("--workload", default="fixed", choices=["fixed", "varlen", "emotion"],
                    help="fixed: configs[1] (8 s pairs, the metric); varlen: configs[4] (3-12 s length-bucketed "
                         "pairs, MUSAN-style noise of its own length, SNR {4, 8}); emotion: configs[3] (dimensional "
                         "emotion head over the frozen encoder, 36 x 5 s)")
    ap.add_argument("--wire", default="f32", choices=["f32", "bf16"],
                    help="gradient all-reduce wire dtype for N > 1 (f32: the exact sum; bf16: half the xGMI bytes)")
    args = ap.parse_args()

    if args.workload == "emotion":
        return bench_emotion(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no torchrun around us: become the launcher (nothing has touched the GPU yet)
        sys.exit(launch_ranks(args.gpus))

    from nrse_amd import arch as A, ddp, kernels as K
    from nrse_amd.engine import ByolEngine, StepConfig, compute_mode

    rank, world, local = ddp.init_from_env()
    if world != args.gpus:
        print(f"error: --gpus {args.gpus} but the launched world has WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    arch = A.LARGE
    B = args.batch
    L = int(args.seconds * 16000)

    # synthetic pairs resident in HBM: clean ~ N(0, 0.1^2), noise ~ N(0, 1), SNR from the YAML
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + 1000 * rank)
    clean_raw = torch.randn(B, L, device=dev, generator=gen) * 0.1
    noise_raw = torch.randn(B, L, device=dev, generator=gen)
    noise_len = torch.full((B,), L, device=dev, dtype=torch.int32)
    snr = torch.tensor([SNR_RANGE[(i + rank) % len(SNR_RANGE)] for i in range(B)], device=dev, dtype=torch.float32)
    clean_iv = torch.empty(B, L, device=dev)
    noisy_iv = torch.empty(B, L, device=dev)
    status = torch.empty(B, device=dev, dtype=torch.int32)
    kscale = torch.empty(B, device=dev)
    total_steps = 1_000_000

    def lr_at(step):  # CosineAnnealingLR(T_max) stepped per iteration (train_byol.py:149-150)
        return 0.5 * 1e-5 * (1 + math.cos(math.pi * step / total_steps))

    varlen_batches = None
    if args.workload == "varlen":
        # configs[4]: every step a different length-bucketed batch of 3-12 s pairs, all staged in
        # HBM before the timed region (the raw mix inputs; the SNR mix runs inside the step)
        from nrse_amd import data as D
        n_items = max(64, (args.steps + args.warmup) * B * world * 2)
        ds = D.SyntheticVarLenPairs(n_items, 16000, 3.0, 12.0, [4, 8], seed=1234)
        dl = D.create_varlen_loader(ds, B, seed=1234, rank=rank, world=world, num_workers=0)
        varlen_batches = []
        for raw in dl:
            varlen_batches.append({k: v.to(dev) for k, v in raw.items()})
            if len(varlen_batches) == args.steps + args.warmup:
                break
        if len(varlen_batches) < args.steps + args.warmup:
            raise SystemExit("varlen: not enough bucketed batches for the requested steps")

    def make_engine(mode):
        cdt, wsplit = compute_mode(mode)
        # fused_zero_grad: the AdamW pass clears the gradient for the next step (no fill kernel)
        eng = ByolEngine(arch, 1024, 2048, device=dev, compute_dtype=cdt, seed=1234, weight_split=wsplit,
                         step_cfg=StepConfig(ema_decay=0.997, overlap_optimizer=not args.serial_optimizer,
                                             fused_zero_grad=os.environ.get("NRSE_FUSED_ZERO_GRAD", "1") != "0"))
        return eng, cdt

    def make_step(eng):
        if varlen_batches is None:
            def step(i):
                K.snr_mix(clean_raw, noise_raw, noise_len, snr, clean_iv, noisy_iv, status, kscale, K.SNR_PEAK_ZMUV)
                return eng.train_step(clean_iv, noisy_iv, lr=lr_at(i), step_seed=i, rank=rank, allreduce=allreduce,
                                      world_size=world)
            return step

        def step(i):  # noqa: F811
            r = varlen_batches[i % len(varlen_batches)]
            Lb = r["clean"].shape[1]
            c = torch.empty(B, Lb, device=dev)
            n = torch.empty(B, Lb, device=dev)
            K.snr_mix(r["clean"], r["noise"], r["noise_len"], r["snr"].float(), c, n, status, kscale, K.SNR_PEAK_ZMUV)
            return eng.train_step(c, n, lr=lr_at(i), step_seed=i, rank=rank, allreduce=allreduce, world_size=world)
        return step

    def serial_probe(eng, step, i):
        """Roofline probe: the timed region runs GEMMs on up to three streams at once, so its event
        durations include time shared with the other streams' kernels. One extra step after the
        timed region runs with the streams serialised (target view, weight gradients and the
        optimizer on the main stream) and brackets every GEMM launch with HIP events on its launch
        stream: per-launch durations of the kernels alone, whose sum stays below the step time."""
        from nrse_amd import engine as E
        serial_prev, overlap_prev = E._SERIAL_TARGET, eng.cfg.overlap_optimizer
        E._SERIAL_TARGET, eng.cfg.overlap_optimizer = True, False
        eng.sync_optimizer()
        torch.cuda.synchronize()
        sprobe = []
        ts0 = time.perf_counter()
        K.set_gemm_probe(sprobe)
        step(i)
        K.set_gemm_probe(None)
        torch.cuda.synchronize()
        sdt_ms = (time.perf_counter() - ts0) * 1e3
        sbytes = K.gemm_probe_bytes()
        E._SERIAL_TARGET, eng.cfg.overlap_optimizer = serial_prev, overlap_prev
        s_gflops = sum(f for f, _, _, _ in sprobe)
        s_ms = sum(e0.elapsed_time(e1) for _, e0, e1, _ in sprobe)
        return dict(gflops=s_gflops, ms=s_ms, bytes=sum(sbytes), launches=len(sprobe), step_ms=sdt_ms, probe=sprobe)

    def timed(eng, step):
        """W untimed warm-up steps, then EXACTLY K steps bracketed by a barrier + device sync on both
        sides (max over ranks for N > 1)."""
        for i in range(args.warmup):
            step(i)
        torch.cuda.synchronize()
        # N > 1: events around each step's all-reduce wait (end of backward -> every exchange done)
        eng.ar_timing = world > 1
        eng.ar_events = []
        executed = [0, 0]
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sent = 0
        for i in range(args.steps):
            step(args.warmup + i)
            executed[0] += eng.executed_layers[0]
            executed[1] += eng.executed_layers[1]
            sent += allreduce.issued_elems if allreduce is not None else 0
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        dt = time.perf_counter() - t0
        return dt, executed, sent

    allreduce = (ddp.GradAllReduce(wire_dtype=torch.bfloat16 if args.wire == "bf16" else None)
                 if world > 1 else None)
    eng, cdt = make_engine(args.dtype)
    step = make_step(eng)
    dt, executed, sent = timed(eng, step)
    ddp_stats = None
    if world > 1:
        # multi-rank readiness record: each rank's time per step, the exposed
        # all-reduce wait (last backward kernel -> all exchanges done, device events on the main
        # stream), and the bytes the gradient exchange puts on the wire per step
        exposed = [e0.elapsed_time(e1) for e0, e1 in eng.ar_events]
        eng.ar_timing = False
        mine = torch.tensor([dt / args.steps * 1e3, sum(exposed) / max(len(exposed), 1)], device=dev, dtype=torch.float64)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        torch.distributed.all_gather(allr, mine)
        esz = 2 if args.wire == "bf16" else 4
        buf_bytes = sent * esz // args.steps   # LayerDrop-skipped layers are not sent
        ddp_stats = {"rank_ms_per_step": [round(float(t[0]), 2) for t in allr],
                     "allreduce_exposed_ms": [round(float(t[1]), 3) for t in allr],
                     "wire": args.wire, "grad_bytes_per_step": buf_bytes,
                     "ring_bytes_per_rank_per_step": int(2 * (world - 1) / world * buf_bytes),
                     "backend": torch.distributed.get_backend()}
        tt = torch.tensor([dt], device=dev)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        dt = float(tt)
    # In-step GEMM durations: one extra step after the timed region, streams overlapped as in the
    # timed steps, with HIP events around every GEMM launch (kept out of the timed region: the
    # event records cost ~2 % of a step when every launch is bracketed)
    probe = []
    tp0 = time.perf_counter()
    K.set_gemm_probe(probe)
    step(args.warmup + args.steps)
    K.set_gemm_probe(None)
    torch.cuda.synchronize()
    probe_step_ms = (time.perf_counter() - tp0) * 1e3
    loss = float(eng.loss_buf)
    st_ok = int((status == 0).sum())
    sp = serial_probe(eng, step, args.warmup + args.steps + 1)
    s_gflops, s_ms, sdt_ms = sp["gflops"], sp["ms"], sp["step_ms"]
    # live roofline of the dominant kernel family (nrse_gemm, MFMA-bound)
    gflops = sum(f for f, _, _, _ in probe)
    gms = sum(e0.elapsed_time(e1) for _, e0, e1, _ in probe)
    n_launch = len(probe)
    achieved_tfs = gflops / (gms * 1e-3) / 1e12 if gms > 0 else 0.0
    if args.detail and rank == 0:
        # per GEMM shape: the in-step (overlapped) and the serial-probe durations
        out = {}
        for tag, pr in (("in_step", probe), ("serial", sp["probe"])):
            per = {}
            for f, e0, e1, shp in pr:
                k = str(shp)
                d = per.setdefault(k, [0.0, 0.0, 0])
                d[0] += f; d[1] += e0.elapsed_time(e1); d[2] += 1
            out[tag] = {k: {"tflops": v[0] / (v[1] * 1e-3) / 1e12, "ms_total": v[1], "launches": v[2]}
                        for k, v in sorted(per.items(), key=lambda kv: -kv[1][1])}
        with open(args.detail, "w") as fh:
            json.dump(out, fh, indent=1)
    avg_exec = (executed[0] / args.steps, executed[1] / args.steps)
    if varlen_batches is None:
        fpp, _ = flops_per_pair(arch, L, avg_exec)
        audio_s = B * L / 16000.0 * args.steps
    else:
        lens = [varlen_batches[args.warmup + i]["clean"].shape[1] for i in range(args.steps)]
        fpp = sum(flops_per_pair(arch, Lb, avg_exec)[0] for Lb in lens) / len(lens)
        audio_s = sum(float(varlen_batches[args.warmup + i]["lengths"].sum()) for i in range(args.steps)) / 16000.0
    pairs = B * world * args.steps
    value = pairs / dt
    peak = BF16_DENSE_PEAK_TFS if cdt == torch.bfloat16 else F32_MFMA_PEAK_TFS
    s_achieved = s_gflops / (s_ms * 1e-3) / 1e12 if s_ms > 0 else 0.0
    result = {
        "metric": ("BYOL utterance-pairs/sec, WavLM-large, 8s@16kHz, batch=32 per GPU" if varlen_batches is None else
                   "BYOL utterance-pairs/sec, WavLM-large, 3-12s@16kHz length-bucketed, batch=32 per GPU"),
        "value": round(value, 3), "unit": "pairs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 2), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": args.dtype, "data": "synthetic (N(0,0.1^2) speech, N(0,1) noise, on-GPU SNR "
                                                         "mix), random-init WavLM-Large weights",
        "config": ({"workload": "configs[1]: WavLM-large BYOL train step, synthetic 8s@16kHz clean/noisy pairs, "
                                "batch=32 per GPU", "global_batch": B * world, "seq_len": L, "frames": arch.frames(L),
                    "parallelism": f"dp{world}", "layerdrop_executed_layers": avg_exec,
                    "grad_wire": args.wire if world > 1 else None}
                   if varlen_batches is None else
                   {"workload": "configs[4]: WavLM-large BYOL, synthetic 3-12 s pairs in 1 s length buckets (padded "
                                "to 0.5 s), noise of independent length tiled on GPU, SNR {4,8} dB, batch=32 per GPU",
                    "global_batch": B * world, "parallelism": f"dp{world}", "layerdrop_executed_layers": avg_exec,
                    "audio_seconds_per_s_per_rank": round(audio_s / dt, 1)}),
        "roofline": {"bound": "mfma", "kernel": "nrse_gemm (every GEMM launch of one step, streams serialised: "
                                                "the probe after the timed region)",
                     "achieved": round(s_achieved, 1), "peak": peak, "unit": "TFLOP/s",
                     "frac": round(s_achieved / peak, 4),
                     "traffic": gemm_traffic(), "traffic_unit": f"HBM bytes per GEMM launch (PMC, profiles/{TRAFFIC_FILE})",
                     "algorithmic_bytes_per_launch": round(sp["bytes"] / max(sp["launches"], 1)),
                     "avg_launch_ms": round(s_ms / max(sp["launches"], 1), 4), "launches": sp["launches"],
                     "gemm_tflop_per_step": round(s_gflops / 1e12, 3), "gemm_ms_per_step": round(s_ms, 3),
                     "probe_step_ms": round(sdt_ms, 2), "gemm_share_of_step": round(s_ms / sdt_ms, 3),
                     "mfma_busy_pmc": gemm_mfma_busy(),
                     "in_step_events": {"achieved": round(achieved_tfs, 1), "frac": round(achieved_tfs / peak, 4),
                                        "launches": n_launch, "avg_launch_ms": round(gms / max(n_launch, 1), 4),
                                        "note": "events around every GEMM of one step run after the timed region with "
                                                "the timed steps' stream overlap; durations include time shared with "
                                                "concurrent streams",
                                        "gemm_share_of_step": round(gms / probe_step_ms, 3)}},
        "step_tflops": round(fpp * value / world / 1e12, 1),
        **({"ddp": ddp_stats} if ddp_stats is not None else {}),
        "loss_last": round(loss, 5), "snr_mix_ok": st_ok,
    }
    if (world == 1 and varlen_batches is None and args.dtype == "bf16" and not args.no_north_star):
        # the north-star mode (embeddings within 1e-3 of the reference) timed by the
        # same process, same steps and warm-up, after the metric's bf16 run
        del eng, step, probe
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        eng2, _ = make_engine("bf16sw")
        step2 = make_step(eng2)
        dt2, executed2, _ = timed(eng2, step2)
        sp2 = serial_probe(eng2, step2, args.warmup + args.steps)
        a2 = sp2["gflops"] / (sp2["ms"] * 1e-3) / 1e12 if sp2["ms"] > 0 else 0.0
        result["north_star_mode"] = {
            "dtype": "bf16sw", "value": round(pairs / dt2, 3), "unit": "pairs/s",
            "ms_per_step": round(dt2 / args.steps * 1e3, 2), "steps": args.steps, "warmup": args.warmup,
            "what": "bf16 activations; forward GEMMs against the split weight: bf16 hi plane + the fp8 correction "
                    "x8 (w - w_hi)8 2^-e on the MX-scaled fp8 MFMA (layers' QKV / FFN), bf16 lo plane elsewhere "
                    "(DESIGN.md §6)" if eng2.online_lo8 is not None else
                    "bf16 activations; forward GEMMs against the split hi + lo bf16 weight planes (DESIGN.md §6)",
            "roofline": {"bound": "mfma", "achieved": round(a2, 1), "peak": BF16_DENSE_PEAK_TFS, "unit": "TFLOP/s",
                         "frac": round(a2 / BF16_DENSE_PEAK_TFS, 4), "launches": sp2["launches"],
                         "gemm_tflop_per_step_bf16_equivalent": round(sp2["gflops"] / 1e12, 3),
                         "gemm_ms_per_step": round(sp2["ms"], 3), "probe_step_ms": round(sp2["step_ms"], 2),
                         "note": "serial probe as the main line's; fp8 segments count half their FLOPs (2x the bf16 "
                                 "MFMA rate)"},
            "parity_vs_reference": north_star_parity(),
            "loss_last": round(float(eng2.loss_buf), 5),
        }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(A.LARGE)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
