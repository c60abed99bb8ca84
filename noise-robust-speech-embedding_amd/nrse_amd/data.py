"""Data side of the BYOL step: noise augmentation on the GPU and the pair loaders.

Reference: src/data/augment.py:4-66 (add_noise_to_speech), src/data/noisy_speech_dataset.py
(NoiseRobustSpeechDataset.__getitem__ :54-148, create_dataloaders :151-194),
src/utils/audio_utils.py (load_and_process_audio :9-64, get_audio_files :67-73).

MI355X design: CPU workers only decode and crop raw waveforms; the SNR mix, the validity checks,
peak normalisation and feature-extractor normalisation run for the whole batch in one fused
kernel (nrse_snr_mix) on the device, producing the dict batches the training loop consumes.
Audio decoding uses the stdlib `wave` reader (PCM WAV) and a restated torchaudio sinc resampler
(nrse_amd/audio.py); torchaudio is not in this image, so `.flac` / `.mp3` files are discovered as
in the reference but take its load-error path (logged, `None`, retry).
"""
from __future__ import annotations

import functools
import os
import random

import logging

import numpy as np
import torch

from . import kernels as K

logger = logging.getLogger("nrse")
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
# decoding / resampling / discovery: nrse_amd/audio.py (audio_utils.py:9-73)
from .audio import (AudioDecodeError, audio_info, check_decodable, get_audio_files, load_audio,  # noqa: E402,F401
                    read_wav)


def crop_or_pad(x: np.ndarray, n: int, rng=random, random_crop: bool = True) -> np.ndarray:
    """Random crop if longer, zero-pad at the end if shorter (audio_utils.py:38-49). `rng` is the
    global `random` module by default, as in the reference (torch's DataLoader reseeds it per
    worker and per epoch)."""
    if x.shape[0] > n:
        start = rng.randint(0, x.shape[0] - n) if random_crop else 0
        return x[start:start + n]
    if x.shape[0] < n:
        return np.pad(x, (0, n - x.shape[0]))
    return x


def audio_valid(x) -> bool:
    """load_and_process_audio's output checks (audio_utils.py:51-58): no NaN, max|x| >= 1e-8."""
    return x is not None and not bool(np.isnan(x).any()) and float(np.max(np.abs(x))) >= 1e-8


MAX_ATTEMPTS = 5   # noisy_speech_dataset.py:56


class WavPairs(torch.utils.data.Dataset):
    """Raw (clean, noise, snr) items from directories of PCM WAV files, with the reference's
    retry rules for invalid audio (noisy_speech_dataset.py:56-76): an invalid clean file moves on
    to the next file, an invalid noise file draws another. Mix failures are detected on the GPU
    (nrse_snr_mix status) and re-drawn by MixedLoader through `redraw` (:80-86, 94-100)."""

    def __init__(self, clean_files, noise_files, sample_rate, max_audio_length, snr_range):
        check_decodable(clean_files, "clean speech files")
        check_decodable(noise_files, "noise files")
        self.clean_files = clean_files
        self.noise_files = noise_files
        self.sr = sample_rate
        self.n = int(max_audio_length * sample_rate)
        self.snr_range = list(snr_range)

    def __len__(self):
        return len(self.clean_files)

    def _load(self, path):
        try:
            x = load_audio(path, self.sr)   # decode, mono, resample (audio_utils.py:26-36)
        except Exception as e:   # audio_utils.py:62-64: load errors -> None
            logger.error(f"Error loading audio file {path}: {e}")
            return None
        x = crop_or_pad(x, self.n)
        return x if audio_valid(x) else None

    def _noise(self):
        return self._load(self.noise_files[random.randint(0, len(self.noise_files) - 1)])

    def __getitem__(self, idx):
        for attempt in range(MAX_ATTEMPTS):
            clean = self._load(self.clean_files[idx])
            if clean is None:
                logger.warning(f"Invalid clean speech file, trying next (attempt {attempt + 1})")
                idx = (idx + 1) % len(self.clean_files)
                continue
            noise = self._noise()
            if noise is None:
                logger.warning(f"Invalid noise file, trying another (attempt {attempt + 1})")
                continue
            return _raw_item(clean, noise, random.choice(self.snr_range), idx, attempt + 1)
        raise RuntimeError(f"no valid pair for item {idx} after {MAX_ATTEMPTS} attempts")

    def redraw(self, idx: int):
        """A fresh noise file and SNR for clean item idx (the reference's `continue` after a
        failed mix keeps idx), or None if the noise file is invalid."""
        clean = self._load(self.clean_files[idx])
        noise = self._noise()
        if clean is None or noise is None:
            return None
        return _raw_item(clean, noise, random.choice(self.snr_range), idx, 0)


def _raw_item(clean, noise, snr, idx, attempts):
    clean = torch.as_tensor(np.ascontiguousarray(clean), dtype=torch.float32)
    noise = torch.as_tensor(np.ascontiguousarray(noise), dtype=torch.float32)
    return {"clean": clean, "noise": noise, "noise_len": torch.tensor(noise.shape[0], dtype=torch.int32),
            "snr": torch.tensor(int(snr), dtype=torch.int64), "index": torch.tensor(idx, dtype=torch.int64),
            "attempts": torch.tensor(attempts, dtype=torch.int32)}


class SyntheticPairs(torch.utils.data.Dataset):
    """Synthetic raw pairs (speech ~ N(0, 0.1^2), noise ~ N(0, 1)), used offline and by bench;
    item idx is a pure function of (seed, idx). `redraw` draws a fresh noise and SNR from the
    global `random` stream."""

    def __init__(self, n_items, samples, snr_range, seed=1234):
        self.n_items, self.samples, self.snr_range, self.seed = n_items, samples, list(snr_range), seed

    def __len__(self):
        return self.n_items

    def _clean(self, idx):
        g = torch.Generator().manual_seed(self.seed * 1000003 + idx)
        return torch.randn(self.samples, generator=g) * 0.1, g

    def __getitem__(self, idx):
        clean, g = self._clean(idx)
        return _raw_item(clean, torch.randn(self.samples, generator=g), self.snr_range[idx % len(self.snr_range)],
                         idx, 1)

    def redraw(self, idx: int):
        clean, _ = self._clean(idx)
        g = torch.Generator().manual_seed(random.getrandbits(62))
        return _raw_item(clean, torch.randn(self.samples, generator=g), random.choice(self.snr_range), idx, 0)


class MockPairs(torch.utils.data.Dataset):
    """configs[0]'s mock data (test/create_mock_dataset.py:4-25) at waveform length: clean ~ N(0, 1),
    SNR cycling through snr_range by index, noisy = clean + N(0, 1) / (snr + 1). Items are already
    the reference's dict batch entries (no mix), as the mock dataset's pairs are."""

    def __init__(self, n_items, samples, snr_range, seed=42):
        g = torch.Generator().manual_seed(seed)
        self.clean = torch.randn(n_items, samples, generator=g)
        self.snrs = torch.tensor([snr_range[i % len(snr_range)] for i in range(n_items)])
        self.noisy = self.clean + torch.randn(n_items, samples, generator=g) / (self.snrs[:, None].float() + 1.0)

    def __len__(self):
        return self.clean.shape[0]

    def __getitem__(self, idx):
        return {"clean_input_values": self.clean[idx][None], "noisy_input_values": self.noisy[idx][None],
                "snr": self.snrs[idx]}


class MixedLoader:
    """Iterable over a DataLoader of raw batches that yields the reference's dict batches
    {clean_input_values [B, 1, L], noisy_input_values [B, 1, L], snr [B]} (noisy_speech_dataset.py:
    140-144, collated), the mix done on the GPU for the whole batch (nrse_snr_mix).

    Failed mixes (the reference's None / `continue` cases, status != 0) are re-drawn with a fresh
    noise and SNR for the same clean item, up to MAX_ATTEMPTS attempts in total per item as in
    the reference, and the batch rows replaced. The status check needs the status on the host:
    batch i+1's mix is enqueued before batch i is handed out, and batch i's status read then, so
    the host waits only for batch i's mix kernel, never for the training step in flight."""

    def __init__(self, raw_loader, dataset, device, do_normalize: bool = True):
        self.raw = raw_loader
        self.dataset = dataset
        self.mixer = GpuMixer(device, do_normalize)
        self.redraws = 0

    def __len__(self):
        return len(self.raw)

    @property
    def sampler(self):
        return self.raw.sampler

    def _enqueue(self, raw):
        batch = self.mixer(raw)
        host = torch.empty(batch["status"].shape, dtype=torch.int32, pin_memory=True)
        host.copy_(batch["status"], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return raw, batch, host, ev

    def _finalize(self, pending):
        raw, batch, host, ev = pending
        ev.synchronize()
        bad = [i for i, st in enumerate(host.tolist()) if st != STATUS_OK]
        attempts = raw.get("attempts", torch.ones(len(host), dtype=torch.int32)).tolist()
        snr = batch["snr"].clone()
        while bad:
            items, rows = [], []
            for i in bad:
                if attempts[i] >= MAX_ATTEMPTS:
                    raise RuntimeError(f"noise mix failed {MAX_ATTEMPTS} times for item "
                                       f"{int(raw['index'][i]) if 'index' in raw else i} (status {int(host[i])})")
                logger.warning(f"Noise addition failed (status {int(host[i])}), trying again "
                               f"(attempt {attempts[i] + 1})")
                it = self.dataset.redraw(int(raw["index"][i]))
                attempts[i] += 1
                if it is None:
                    continue
                items.append(it)
                rows.append(i)
            if not items:
                continue
            L = batch["clean_input_values"].shape[-1]
            Ln = max(int(it["noise"].shape[0]) for it in items)
            sub = {"clean": torch.stack([torch.nn.functional.pad(it["clean"][:L], (0, L - min(L, it["clean"].shape[0])))
                                         for it in items]),
                   "noise": torch.stack([torch.nn.functional.pad(it["noise"], (0, Ln - it["noise"].shape[0]))
                                         for it in items]),
                   "noise_len": torch.stack([it["noise_len"] for it in items]),
                   "snr": torch.stack([it["snr"] for it in items])}
            mixed = self.mixer(sub)
            st = mixed["status"].tolist()
            self.redraws += len(items)
            idx = torch.tensor(rows, device=batch["clean_input_values"].device)
            batch["clean_input_values"].index_copy_(0, idx, mixed["clean_input_values"])
            batch["noisy_input_values"].index_copy_(0, idx, mixed["noisy_input_values"])
            for r, s_, it in zip(rows, st, items):
                snr[r] = it["snr"]
            bad = [r for r, s_ in zip(rows, st) if s_ != STATUS_OK] + [i for i in bad if i not in rows]
        return {"clean_input_values": batch["clean_input_values"], "noisy_input_values": batch["noisy_input_values"],
                "snr": snr}

    def __iter__(self):
        pending = None
        for raw in self.raw:
            cur = self._enqueue(raw)
            if pending is not None:
                yield self._finalize(pending)
            pending = cur
        if pending is not None:
            yield self._finalize(pending)


def _rank_share(ds, rank: int, world: int):
    """Equal, disjoint per-rank shares: truncate to world * floor(N / world), then stride, so
    every rank sees the same number of batches (no rank blocks in an all-reduce another rank
    never issues) and the same LR schedule length."""
    if world <= 1:
        return ds
    n = (len(ds) // world) * world
    return torch.utils.data.Subset(ds, list(range(rank, n, world)))


def rank_generator(seed: int, rank: int) -> torch.Generator:
    """The DataLoader's generator, distinct per rank. torch derives each worker's `random` /
    torch seeds (base_seed + worker_id) from it, so with a per-rank generator the noise file,
    SNR and crop draws of item k differ across ranks (the same torch.manual_seed on every rank
    would otherwise repeat them rank to rank). With num_workers = 0 the items draw from the main
    process's `random`, seeded per rank by `seed_host_rng`."""
    return torch.Generator().manual_seed(int(seed) * 1000003 + 7919 * int(rank) + 1)


def seed_host_rng(seed: int, rank: int) -> None:
    """Seed the main process's `random` per rank (item draws at num_workers = 0, MixedLoader's
    redraws); src/utils/setup_utils.py:4-7 seeds torch and numpy but not `random`."""
    random.seed(int(seed) * 1000003 + 7919 * int(rank))


def create_raw_dataloaders(config: dict, *, synthetic_items: int | None = None, rank: int = 0, world: int = 1):
    """(train_loader, val_loader, base dataset) of RAW batches, split with the seeded generator as
    in create_dataloaders (noisy_speech_dataset.py:163-175).

    Data: the WAV files under `data.clean_data_path` / `data.noise_data_path`; a directory that is
    missing or holds no audio file raises (a mistyped path must not train on anything else).
    Synthetic pairs only when asked for explicitly: `synthetic_items=N` or `data.synthetic: N`.

    Batching follows the reference's DataLoaders (noisy_speech_dataset.py:178-192): no drop_last,
    so len(loader) = ceil(items / batch_size) and the validation tail is kept. One guard: a final
    TRAINING batch of exactly one pair is dropped -- the heads' BatchNorm1d in train mode cannot
    normalise a single row (the reference raises "Expected more than 1 value per channel" there,
    SURVEY.md §4)."""
    d, t = config["data"], config["training"]
    sr, secs = int(d["sample_rate"]), float(d["max_audio_length"])
    synthetic = synthetic_items or int(d.get("synthetic", 0) or 0)
    if synthetic:
        ds = SyntheticPairs(int(synthetic), int(sr * secs), d["snr_range"], seed=t.get("seed", 42))
    else:
        files = {}
        for key in ("clean_data_path", "noise_data_path"):
            path = d.get(key, "")
            if not path or not os.path.isdir(path):
                raise FileNotFoundError(f"data.{key} = {path!r} is not a directory (set data.synthetic: N for "
                                        f"synthetic pairs)")
            files[key] = get_audio_files(path)
            if not files[key]:
                raise FileNotFoundError(f"data.{key} = {path!r} holds no .wav/.flac/.mp3 file")
        ds = WavPairs(files["clean_data_path"], files["noise_data_path"], sr, secs, d["snr_range"])
    val_size = int(len(ds) * d.get("validation_ratio", 0.1))
    train_ds, val_ds = torch.utils.data.random_split(
        ds, [len(ds) - val_size, val_size], generator=torch.Generator().manual_seed(t.get("seed", 42)))
    train_ds, val_ds = _rank_share(train_ds, rank, world), _rank_share(val_ds, rank, world)
    bs = int(t["batch_size"])
    kw = dict(batch_size=bs, num_workers=min(int(t.get("num_workers", 4)), 8), pin_memory=True)
    seed = int(t.get("seed", 42))
    train = torch.utils.data.DataLoader(train_ds, shuffle=True, generator=rank_generator(seed, rank),
                                        drop_last=bs > 1 and len(train_ds) % bs == 1, **kw)
    val = (torch.utils.data.DataLoader(val_ds, shuffle=False, generator=rank_generator(seed + 1, rank),
                                       drop_last=False, **kw)
           if len(val_ds) > 0 else None)
    return train, val, ds


def create_dataloaders(config: dict, feature_extractor=None, *, device=None, synthetic_items: int | None = None,
                       rank: int = 0, world: int = 1):
    """Drop-in for create_dataloaders (noisy_speech_dataset.py:151-194): (train_loader,
    val_loader) yielding the reference's dict batches, mixed and normalised on the GPU.
    `feature_extractor` is accepted for signature compatibility; its normalisation is
    `config['data']['do_normalize']` (default True, Wav2Vec2FeatureExtractor's). The optional
    `config['data']['mock_items']` selects configs[0]'s mock dataset (MockPairs)."""
    d, t = config["data"], config["training"]
    if d.get("mock_items"):
        ds = MockPairs(int(d["mock_items"]), int(int(d["sample_rate"]) * float(d["max_audio_length"])),
                       d["snr_range"], seed=t.get("seed", 42))
        val_size = int(len(ds) * d.get("validation_ratio", 0.1))
        tr, va = torch.utils.data.random_split(ds, [len(ds) - val_size, val_size],
                                               generator=torch.Generator().manual_seed(t.get("seed", 42)))
        tr, va = _rank_share(tr, rank, world), _rank_share(va, rank, world)
        bs = int(t["batch_size"])
        # pinned batches: the loop's .to(device, non_blocking=True) is then an async DMA copy
        pin = torch.cuda.is_available()
        return (torch.utils.data.DataLoader(tr, shuffle=True, batch_size=bs, num_workers=0, pin_memory=pin,
                                            drop_last=bs > 1 and len(tr) % bs == 1),
                torch.utils.data.DataLoader(va, shuffle=False, batch_size=bs, num_workers=0, pin_memory=pin)
                if len(va) > 0 else None)
    if feature_extractor is not None and hasattr(feature_extractor, "do_normalize"):
        d = {**d, "do_normalize": bool(feature_extractor.do_normalize)}
    device = device or torch.device("cuda", torch.cuda.current_device())
    train, val, base = create_raw_dataloaders(config, synthetic_items=synthetic_items, rank=rank, world=world)
    norm = d.get("do_normalize", True)
    return MixedLoader(train, base, device, norm), (MixedLoader(val, base, device, norm) if val is not None else None)


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
            "snr": torch.stack([it["snr"] for it in items]), "lengths": torch.tensor(lens, dtype=torch.int64),
            **({"index": torch.stack([it["index"] for it in items]),
                "attempts": torch.stack([it["attempts"] for it in items])} if "index" in items[0] else {})}


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
        clean = torch.randn(int(self.lengths[idx]), generator=g) * 0.1
        return _raw_item(clean, torch.randn(int(self.noise_lengths[idx]), generator=g),
                         self.snr_range[idx % len(self.snr_range)], idx, 1)

    def redraw(self, idx: int):
        g = torch.Generator().manual_seed(self.seed * 1000003 + idx)
        clean = torch.randn(int(self.lengths[idx]), generator=g) * 0.1
        g2 = torch.Generator().manual_seed(random.getrandbits(62))
        return _raw_item(clean, torch.randn(int(self.noise_lengths[idx]), generator=g2), random.choice(self.snr_range),
                         idx, 0)


def wav_num_samples(path: str, sample_rate: int | None = None) -> int:
    """Samples of `path` after resampling to `sample_rate` (torchaudio's ceil(new * n / orig))."""
    n, sr = audio_info(path)
    if sample_rate is None or sr == sample_rate:
        return n
    g = np.gcd(sr, sample_rate)
    return -(-(sample_rate // g) * n // (sr // g))


class WavVarLenPairs(torch.utils.data.Dataset):
    """Clean files at their own length (cropped to max_s), noise from a pool (MUSAN). Files the
    build cannot decode (or whose header is broken) are logged and left out of the clean list
    (their length, which the bucketing needs, is unknown); undecodable noise files take the
    reference's retry path."""

    def __init__(self, clean_files, noise_files, sample_rate, max_s, snr_range):
        check_decodable(clean_files, "clean speech files")
        check_decodable(noise_files, "noise files")
        self.sr, self.nmax = sample_rate, int(max_s * sample_rate)
        self.snr_range = list(snr_range)
        self.clean_files, self.lengths = [], []
        for f in clean_files:
            try:
                n = wav_num_samples(f, sample_rate)
            except Exception as e:
                logger.error(f"Error loading audio file {f}: {e}")
                continue
            self.clean_files.append(f)
            self.lengths.append(min(n, self.nmax))
        self.noise_files = noise_files

    def __len__(self):
        return len(self.clean_files)

    def _load(self, path, crop: bool):
        try:
            x = load_audio(path, self.sr)
        except Exception as e:   # audio_utils.py:62-64
            logger.error(f"Error loading audio file {path}: {e}")
            return None
        x = crop_or_pad(x, self.nmax) if (crop and x.shape[0] > self.nmax) else x
        return x if audio_valid(x) else None

    def __getitem__(self, idx):
        # the loader's per-rank, per-worker seeded `random` (create_varlen_loader). The sampler
        # put idx in the bucket of lengths[idx]: a substitute file (an invalid clean file moves
        # on to the next one, noisy_speech_dataset.py:56-66) is cropped / padded to that length,
        # so the batch keeps its padded shape, and the item keeps the sampled index.
        L, idx0 = self.lengths[idx], idx
        for attempt in range(MAX_ATTEMPTS):
            clean = self._load(self.clean_files[idx], True)
            if clean is None:
                logger.warning(f"Invalid clean speech file, trying next (attempt {attempt + 1})")
                idx = (idx + 1) % len(self.clean_files)
                continue
            noise = self._load(self.noise_files[random.randint(0, len(self.noise_files) - 1)], True)
            if noise is None:
                logger.warning(f"Invalid noise file, trying another (attempt {attempt + 1})")
                continue
            clean = crop_or_pad(clean, L, random_crop=False)
            return _raw_item(clean, noise, random.choice(self.snr_range), idx0, attempt + 1)
        raise RuntimeError(f"no valid pair for item {idx0} after {MAX_ATTEMPTS} attempts")


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
                                       pin_memory=True, generator=rank_generator(seed, rank))
