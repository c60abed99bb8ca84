"""Audio file decoding and resampling for the loader workers (reference src/utils/audio_utils.py).

The reference loads with torchaudio (`torchaudio.load`, `torchaudio.transforms.Resample(sr,
sample_rate)`, audio_utils.py:26-36) and discovers `.wav/.flac/.mp3` (:67-73). torchaudio is not
in this image, so:

* decoding: PCM WAV through the stdlib `wave` reader; `.flac` / `.mp3` are discovered like the
  reference but cannot be decoded here -- `load_audio` raises `AudioDecodeError`, which the
  datasets turn into the reference's load-error path (`None`, logged once per file, retry); a
  file list in which more than half the files cannot be decoded is refused up front
  (`check_decodable`), so such a corpus fails loudly instead of training on retries;
* resampling: `resample` restates torchaudio.functional.resample's default method
  (`sinc_interp_hann`, lowpass_filter_width 6, rolloff 0.99; torchaudio 2.x
  `_get_sinc_resample_kernel` / `_apply_sinc_resample_kernel`): a windowed-sinc polyphase filter
  over the rates reduced by their gcd, output length ceil(new * n / orig). Parity is UNPINNED:
  torchaudio is not importable here and the reference ships no resampled fixture; the tests
  check the filter's published properties (DC gain 1, a pure tone below the cut-off keeps its
  frequency and amplitude, identity at equal rates, the output length).
This runs in the CPU DataLoader workers, where the reference runs it too; the SNR mix and the
normalisations stay on the GPU (nrse_snr_mix).
"""
from __future__ import annotations

import logging
import math
import os
import wave
from functools import lru_cache

import numpy as np
import torch

logger = logging.getLogger("nrse")
AUDIO_EXTS = (".wav", ".flac", ".mp3")   # audio_utils.py:69


class AudioDecodeError(RuntimeError):
    pass


def get_audio_files(path: str, exts=AUDIO_EXTS) -> list:
    """audio_utils.py:67-73 (sorted, so every rank and run lists the same files in the same order)."""
    out = []
    for root, _, files in os.walk(path):
        for f in files:
            if os.path.splitext(f)[1].lower() in exts:
                out.append(os.path.join(root, f))
    return sorted(out)


def undecodable_share(files: list, probe: int = 256) -> float:
    """Share of `files` this build cannot decode: every file whose format has no decoder here
    (.flac / .mp3), plus the share of broken WAV headers among up to `probe` evenly spaced WAV
    files (their header is read, not their samples)."""
    if not files:
        return 0.0
    wavs = [f for f in files if os.path.splitext(f)[1].lower() == ".wav"]
    bad = len(files) - len(wavs)
    if wavs:
        step = max(1, len(wavs) // probe)
        sample = wavs[::step]
        broken = 0
        for f in sample:
            try:
                audio_info(f)
            except Exception:
                broken += 1
        bad += broken / len(sample) * len(wavs)
    return bad / len(files)


def check_decodable(files: list, what: str, max_share: float = 0.5) -> None:
    """Refuse a file list mostly made of audio this build cannot decode: the reference decodes
    any torchaudio format (audio_utils.py:27), so a FLAC / MP3 corpus would otherwise train on
    nothing but load errors and retries (noisy_speech_dataset.py:56-76)."""
    share = undecodable_share(files)
    if share > max_share:
        raise AudioDecodeError(
            f"{what}: {share:.0%} of {len(files)} files cannot be decoded by this build (PCM WAV only; "
            f"torchaudio and its codecs are absent). Convert the corpus to WAV.")
    if share > 0:
        logger.warning(f"{what}: {share:.1%} of {len(files)} files cannot be decoded and will take the "
                       f"load-error path")


def read_wav(path: str) -> tuple:
    """PCM WAV -> (mono float32 samples in [-1, 1), sample rate); channels averaged like
    audio_utils.py:27-29."""
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
        raise AudioDecodeError(f"{path}: unsupported sample width {width}")
    if ch > 1:
        x = x.reshape(-1, ch).mean(axis=1)
    return x, sr


def audio_info(path: str) -> tuple:
    """(frames, sample rate) without decoding the samples (WAV only)."""
    if os.path.splitext(path)[1].lower() != ".wav":
        raise AudioDecodeError(f"{path}: no decoder for this format in this build (torchaudio absent)")
    with wave.open(path, "rb") as w:
        return w.getnframes(), w.getframerate()


def load_audio(path: str, sample_rate: int) -> np.ndarray:
    """Decode, mix down to mono and resample to `sample_rate` (audio_utils.py:26-36)."""
    if os.path.splitext(path)[1].lower() != ".wav":
        raise AudioDecodeError(f"{path}: no decoder for this format in this build (torchaudio absent)")
    x, sr = read_wav(path)
    if sr != sample_rate:
        x = resample(x, sr, sample_rate)
    return x


@lru_cache(maxsize=16)
def _sinc_kernel(orig: int, new: int, lowpass_filter_width: int = 6, rolloff: float = 0.99):
    """[new, 1, 2*width + orig] polyphase filter bank (float64 build, float32 result) and width."""
    base = min(orig, new) * rolloff
    width = math.ceil(lowpass_filter_width * orig / base)
    idx = np.arange(-width, width + orig, dtype=np.float64)[None, :] / orig
    t = np.arange(0, -new, -1, dtype=np.float64)[:, None] / new + idx
    t = np.clip(t * base, -lowpass_filter_width, lowpass_filter_width)
    window = np.cos(t * math.pi / lowpass_filter_width / 2) ** 2
    t = t * math.pi
    with np.errstate(invalid="ignore", divide="ignore"):
        k = np.where(t == 0, 1.0, np.sin(t) / t)
    k = k * window * (base / orig)
    return torch.from_numpy(k.astype(np.float32))[:, None, :], width


def resample(x: np.ndarray, orig_freq: int, new_freq: int) -> np.ndarray:
    """torchaudio.functional.resample(x, orig_freq, new_freq) with its defaults (see module doc)."""
    orig_freq, new_freq = int(orig_freq), int(new_freq)
    if orig_freq <= 0 or new_freq <= 0:
        raise ValueError("sample rates must be positive")
    if orig_freq == new_freq:
        return np.asarray(x, np.float32)
    g = math.gcd(orig_freq, new_freq)
    o, n = orig_freq // g, new_freq // g
    kernel, width = _sinc_kernel(o, n)
    w = torch.as_tensor(np.ascontiguousarray(x, np.float32)).reshape(1, 1, -1)
    length = w.shape[-1]
    w = torch.nn.functional.pad(w, (width, width + o))
    out = torch.nn.functional.conv1d(w, kernel, stride=o)          # [1, n, frames]
    out = out.transpose(1, 2).reshape(-1)
    target = math.ceil(n * length / o)
    return out[:target].numpy()
