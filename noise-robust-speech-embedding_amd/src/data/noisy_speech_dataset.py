"""Mirror of reference src/data/noisy_speech_dataset.py: raw-waveform loaders + on-GPU mixing."""
from nrse_amd.data import GpuMixer, SyntheticPairs, WavPairs, create_dataloaders  # noqa: F401
