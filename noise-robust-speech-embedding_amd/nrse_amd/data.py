"""Data side of the BYOL step: noise augmentation on the GPU and the pair loaders.

Reference: src/data/augment.py:4-66 (add_noise_to_speech), src/data/noisy_speech_dataset.py
(NoiseRobustSpeechDataset.__getitem__ :54-148, create_dataloaders :151-194),
src/utils/audio_utils.py (load_and_process_audio :9-64, get_audio_files :67-73).

MI355X design: CPU workers only decode and crop raw waveforms; the SNR mix, the validity checks,
peak normalisation and feature-extractor normalisation run for the whole batch in one fused
kernel (nrse_snr_mix) on the device, producing the dict batches the training loop consumes.
Audio decoding uses the stdlib `wave` reader (PCM WAV); torchaudio is not in this image, so
compressed formats and resampling are not supported (files must be at the configured rate).
"""
from __future__ import annotations

import functools
import os
import random
import wave

import numpy as np
import torch

from . import kernels as K

STATUS_OK = 0


def add_noise_to_speech(speech: torch.Tensor, noise: torch.Tensor, snr_db: float):
    """Drop-in for src/data/augment.py:4: speech [1, L], noise [1, Ln] -> noisy [1, L] or None."""
    dev = speech.device if speech.is_cuda else torch.device("cuda", torch.cuda.current_device())
    s = speech.reshape(1, -1).to(dev, torch.float32).contiguous()
    n = noise.reshape(1, -1).to(dev, torch.float32).contiguous()
    out_c = torch.empty_like(s)
    out_n = torch.empty_like(s)
    status = torch.empty(1, device=dev, dtype=torch.int32)
    nlen = torch.tensor([n.shape[1]], device=dev, dtype=torch.int32)
    snr = torch.tensor([float(snr_db)], device=dev, dtype=torch.float32)
    K.snr_mix(s, n, nlen, snr, out_c, out_n, status, None, K.SNR_RAW)
    if int(status.item()) != STATUS_OK:   # the reference returns None (host decision)
        return None
    return out_n.to(speech.device) if not speech.is_cuda else out_n


class GpuMixer:
    """Raw batch {clean [B, L], noise [B, Ln_max], noise_len [B], snr [B]} -> the reference's dict
    batch {clean_input_values, noisy_input_values [B, 1, L], snr [B]} computed on the device."""

    def __init__(self, device, do_normalize: bool = True):
        self.dev = torch.device(device)
        self.mode = K.SNR_PEAK_ZMUV if do_normalize else K.SNR_PEAK

    def __call__(self, raw: dict) -> dict:
        clean = raw["clean"].to(self.dev, torch.float32, non_blocking=True).contiguous()
        noise = raw["noise"].to(self.dev, torch.float32, non_blocking=True).contiguous()
        nlen = raw["noise_len"].to(self.dev, torch.int32, non_blocking=True)
        snr = raw["snr"].to(self.dev, torch.float32, non_blocking=True)
        B, L = clean.shape
        c = torch.empty(B, L, device=self.dev)
        n = torch.empty(B, L, device=self.dev)
        status = torch.empty(B, device=self.dev, dtype=torch.int32)
        K.snr_mix(clean, noise, nlen, snr, c, n, status, None, self.mode)
        return {"clean_input_values": c.view(B, 1, L), "noisy_input_values": n.view(B, 1, L),
                "snr": raw["snr"].to(torch.int64), "status": status}


# ----------------------------------------------------------------------------- audio files
def get_audio_files(path: str, exts=(".wav",)) -> list:
    out = []
    for root, _, files in os.walk(path):
        for f in sorted(files):
            if f.lower().endswith(exts):
                out.append(os.path.join(root, f))
    return sorted(out)


def read_wav(path: str) -> tuple:
    with wave.open(path, "rb") as w:
        sr, ch, width, n = w.getframerate(), w.getnchannels(), w.getsampwidth(), w.getnframes()
        buf = w.readframes(n)
    if width == 2:
        x = np.frombuffer(buf, dtype="<i2").astype(np.float32) / 32768.0
    elif width == 4:
        x = np.frombuffer(buf, dtype="<i4").astype(np.float32) / 2147483648.0
    elif width == 1:
        x = (np.frombuffer(buf, dtype=np.uint8).astype(np.float32) - 128.0) / 128.0
    else:
        raise ValueError(f"{path}: unsupported sample width {width}")
    if ch > 1:
        x = x.reshape(-1, ch).mean(axis=1)  # mono mix-down (audio_utils.py:27-29)
    return x, sr


def crop_or_pad(x: np.ndarray, n: int, rng: random.Random, random_crop: bool = True) -> np.ndarray:
    """Random crop if longer, zero-pad at the end if shorter (audio_utils.py:38-49)."""
    if x.shape[0] > n:
        start = rng.randint(0, x.shape[0] - n) if random_crop else 0
        return x[start:start + n]
    if x.shape[0] < n:
        return np.pad(x, (0, n - x.shape[0]))
    return x


class WavPairs(torch.utils.data.Dataset):
    """Raw (clean, noise, snr) items from directories of PCM WAV files."""

    def __init__(self, clean_files, noise_files, sample_rate, max_audio_length, snr_range, seed=42):
        self.clean_files = clean_files
        self.noise_files = noise_files
        self.sr = sample_rate
        self.n = int(max_audio_length * sample_rate)
        self.snr_range = list(snr_range)
        self.rng = random.Random(seed)

    def __len__(self):
        return len(self.clean_files)

    def _load(self, path):
        x, sr = read_wav(path)
        if sr != self.sr:
            raise ValueError(f"{path}: sample rate {sr} != {self.sr} (no resampler in this build)")
        return crop_or_pad(x, self.n, self.rng)

    def __getitem__(self, idx):
        clean = self._load(self.clean_files[idx])
        noise = self._load(self.noise_files[self.rng.randint(0, len(self.noise_files) - 1)])
        return {"clean": torch.from_numpy(clean), "noise": torch.from_numpy(noise),
                "noise_len": torch.tensor(noise.shape[0], dtype=torch.int32),
                "snr": torch.tensor(self.rng.choice(self.snr_range), dtype=torch.int64)}


class SyntheticPairs(torch.utils.data.Dataset):
    """Synthetic raw pairs (speech ~ N(0, 0.1^2), noise ~ N(0, 1)), used offline and by bench."""

    def __init__(self, n_items, samples, snr_range, seed=1234):
        self.n_items, self.samples, self.snr_range, self.seed = n_items, samples, list(snr_range), seed

    def __len__(self):
        return self.n_items

    def __getitem__(self, idx):
        g = torch.Generator().manual_seed(self.seed * 1000003 + idx)
        return {"clean": torch.randn(self.samples, generator=g) * 0.1, "noise": torch.randn(self.samples, generator=g),
                "noise_len": torch.tensor(self.samples, dtype=torch.int32),
                "snr": torch.tensor(self.snr_range[idx % len(self.snr_range)], dtype=torch.int64)}


def create_dataloaders(config: dict, feature_extractor=None, *, synthetic_items: int | None = None,
                       rank: int = 0, world: int = 1):
    """(train_loader, val_loader) of RAW batches, split 85/15 with the seeded generator like
    create_dataloaders (noisy_speech_dataset.py:163-175); feed them through GpuMixer."""
    d, t = config["data"], config["training"]
    sr, secs = int(d["sample_rate"]), float(d["max_audio_length"])
    clean_dir, noise_dir = d.get("clean_data_path", ""), d.get("noise_data_path", "")
    if os.path.isdir(clean_dir) and os.path.isdir(noise_dir):
        ds = WavPairs(get_audio_files(clean_dir), get_audio_files(noise_dir), sr, secs, d["snr_range"],
                      seed=t.get("seed", 42) + rank)
    else:
        n = synthetic_items or 64 * int(t["batch_size"])
        ds = SyntheticPairs(n, int(sr * secs), d["snr_range"], seed=t.get("seed", 42))
    val_size = int(len(ds) * d.get("validation_ratio", 0.1))
    train_ds, val_ds = torch.utils.data.random_split(
        ds, [len(ds) - val_size, val_size], generator=torch.Generator().manual_seed(t.get("seed", 42)))
    if world > 1:
        train_ds = torch.utils.data.Subset(train_ds, list(range(rank, len(train_ds), world)))
    kw = dict(batch_size=int(t["batch_size"]), num_workers=min(int(t.get("num_workers", 4)), 8), pin_memory=True,
              drop_last=True)
    train = torch.utils.data.DataLoader(train_ds, shuffle=True, **kw)
    val = torch.utils.data.DataLoader(val_ds, shuffle=False, **kw) if val_size >= int(t["batch_size"]) else None
    return train, val


# ----------------------------------------------------------------------------- variable length
# BASELINE config 5: variable-length 3-12 s utterances in length-bucketed batches. The reference
# crops/pads every item to one fixed length (audio_utils.py:38-49) and its encoder takes no
# attention mask (src/models/encoder.py:23-25); bucketing keeps those semantics per batch (zero
# padding at the end, to the batch's padded length) while cutting the padding work.
def padded_length(n: int, multiple: int) -> int:
    return ((n + multiple - 1) // multiple) * multiple


class LengthBucketBatchSampler(torch.utils.data.Sampler):
    """Batches of indices whose lengths fall in the same bucket (`boundaries`, in samples,
    ascending; bucket i holds lengths in (boundaries[i-1], boundaries[i]]). Seeded per epoch:
    items are shuffled inside buckets, cut into batches, the batch order shuffled, and with
    world > 1 every rank takes an equal, disjoint share of the batches (rank-strided)."""

    def __init__(self, lengths, batch_size: int, boundaries, *, seed: int = 42, rank: int = 0, world: int = 1,
                 drop_last: bool = True):
        self.lengths = [int(n) for n in lengths]
        self.batch_size = int(batch_size)
        self.boundaries = [int(b) for b in boundaries]
        self.seed, self.rank, self.world, self.drop_last = seed, rank, world, drop_last
        self.epoch = 0

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def bucket_of(self, n: int) -> int:
        for i, b in enumerate(self.boundaries):
            if n <= b:
                return i
        return len(self.boundaries)

    def _batches(self) -> list:
        rng = random.Random(self.seed * 1000003 + self.epoch)
        buckets = {}
        for i, n in enumerate(self.lengths):
            buckets.setdefault(self.bucket_of(n), []).append(i)
        batches = []
        for k in sorted(buckets):
            idx = buckets[k]
            rng.shuffle(idx)
            for s in range(0, len(idx), self.batch_size):
                b = idx[s:s + self.batch_size]
                if len(b) == self.batch_size or not self.drop_last:
                    batches.append(b)
        rng.shuffle(batches)
        n = (len(batches) // self.world) * self.world
        return batches[:n][self.rank::self.world]

    def __iter__(self):
        return iter(self._batches())

    def __len__(self) -> int:
        return len(self._batches())


def collate_varlen(items: list, pad_multiple: int = 8000) -> dict:
    """Raw varlen items -> {clean [B, Lp], noise [B, Ln], noise_len [B], snr [B], lengths [B]}:
    clean zero-padded at the end to the batch maximum rounded up to `pad_multiple` samples (a
    bounded set of step shapes), noise zero-padded to its batch maximum (the on-GPU mix tiles
    each noise by its own noise_len, augment.py:10-15)."""
    lens = [int(it["clean"].shape[0]) for it in items]
    Lp = padded_length(max(lens), pad_multiple)
    Ln = max(int(it["noise"].shape[0]) for it in items)
    B = len(items)
    clean = torch.zeros(B, Lp)
    noise = torch.zeros(B, Ln)
    for i, it in enumerate(items):
        clean[i, :lens[i]] = it["clean"]
        noise[i, :it["noise"].shape[0]] = it["noise"]
    return {"clean": clean, "noise": noise,
            "noise_len": torch.tensor([int(it["noise"].shape[0]) for it in items], dtype=torch.int32),
            "snr": torch.stack([it["snr"] for it in items]), "lengths": torch.tensor(lens, dtype=torch.int64)}


class SyntheticVarLenPairs(torch.utils.data.Dataset):
    """Synthetic raw pairs with seeded lengths U[min_s, max_s] seconds (speech ~ N(0, 0.1^2),
    noise ~ N(0, 1) of an independent random length: the MUSAN-style noise pool of config 5)."""

    def __init__(self, n_items, sample_rate, min_s, max_s, snr_range, seed=1234):
        self.n_items, self.sr, self.snr_range, self.seed = n_items, sample_rate, list(snr_range), seed
        g = np.random.default_rng(seed)
        self.lengths = g.integers(int(min_s * sample_rate), int(max_s * sample_rate) + 1, n_items)
        self.noise_lengths = g.integers(int(min_s * sample_rate), int(max_s * sample_rate) + 1, n_items)

    def __len__(self):
        return self.n_items

    def __getitem__(self, idx):
        g = torch.Generator().manual_seed(self.seed * 1000003 + idx)
        return {"clean": torch.randn(int(self.lengths[idx]), generator=g) * 0.1,
                "noise": torch.randn(int(self.noise_lengths[idx]), generator=g),
                "noise_len": torch.tensor(int(self.noise_lengths[idx]), dtype=torch.int32),
                "snr": torch.tensor(self.snr_range[idx % len(self.snr_range)], dtype=torch.int64)}


def wav_num_samples(path: str) -> int:
    with wave.open(path, "rb") as w:
        return w.getnframes()


class WavVarLenPairs(torch.utils.data.Dataset):
    """PCM WAV clean files at their own length (cropped to max_s), noise from a pool (MUSAN)."""

    def __init__(self, clean_files, noise_files, sample_rate, max_s, snr_range, seed=42):
        self.clean_files, self.noise_files = clean_files, noise_files
        self.sr, self.nmax = sample_rate, int(max_s * sample_rate)
        self.snr_range = list(snr_range)
        self.rng = random.Random(seed)
        self.lengths = [min(wav_num_samples(f), self.nmax) for f in clean_files]

    def __len__(self):
        return len(self.clean_files)

    def _load(self, path, crop: bool):
        x, sr = read_wav(path)
        if sr != self.sr:
            raise ValueError(f"{path}: sample rate {sr} != {self.sr} (no resampler in this build)")
        return crop_or_pad(x, self.nmax, self.rng) if (crop and x.shape[0] > self.nmax) else x

    def __getitem__(self, idx):
        clean = self._load(self.clean_files[idx], True)
        noise = self._load(self.noise_files[self.rng.randint(0, len(self.noise_files) - 1)], True)
        return {"clean": torch.from_numpy(np.ascontiguousarray(clean)), "noise": torch.from_numpy(np.ascontiguousarray(noise)),
                "noise_len": torch.tensor(noise.shape[0], dtype=torch.int32),
                "snr": torch.tensor(self.rng.choice(self.snr_range), dtype=torch.int64)}


def create_varlen_loader(dataset, batch_size: int, *, sample_rate: int = 16000, min_s: float = 3.0,
                         max_s: float = 12.0, bucket_s: float = 1.0, pad_s: float = 0.5, seed: int = 42,
                         rank: int = 0, world: int = 1, num_workers: int = 4):
    """DataLoader of length-bucketed raw batches for a dataset exposing `.lengths` (samples)."""
    edges = []
    e = min_s + bucket_s
    while e < max_s + 1e-9:
        edges.append(int(round(e * sample_rate)))
        e += bucket_s
    sampler = LengthBucketBatchSampler(dataset.lengths, batch_size, edges, seed=seed, rank=rank, world=world)
    pad = int(pad_s * sample_rate)
    return torch.utils.data.DataLoader(dataset, batch_sampler=sampler, num_workers=num_workers,
                                       collate_fn=functools.partial(collate_varlen, pad_multiple=pad),
                                       pin_memory=True)
