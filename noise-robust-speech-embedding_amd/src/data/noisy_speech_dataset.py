"""Mirror of reference src/data/noisy_speech_dataset.py (NoiseRobustSpeechDataset :12-148,
create_dataloaders :151-194). create_dataloaders yields the reference's dict batches
{clean_input_values, noisy_input_values, snr}; the mix, the validity checks and the
normalisation run on the GPU per batch (nrse_amd.data.MixedLoader), with the reference's retry
rules."""
from nrse_amd.data import (GpuMixer, MixedLoader, MockPairs, SyntheticPairs, WavPairs,  # noqa: F401
                           create_dataloaders, create_raw_dataloaders, get_audio_files)


class NoiseRobustSpeechDataset(WavPairs):
    """Constructor of the reference dataset (:13-40). Items are raw (clean, noise, snr) waveforms:
    the per-item mix of the reference (:77-129) happens batched on the GPU in MixedLoader."""

    def __init__(self, clean_data_path, noise_data_path, sample_rate=16000, max_audio_length=5.0,
                 snr_range=(0, 5, 10, 15, 20), feature_extractor=None):
        super().__init__(get_audio_files(clean_data_path), get_audio_files(noise_data_path), sample_rate,
                         max_audio_length, snr_range)
        self.feature_extractor = feature_extractor
        print(f"Found {len(self.clean_files)} clean files and {len(self.noise_files)} noise files.")
