"""Mirror of reference src/data/noisy_speech_dataset.py (NoiseRobustSpeechDataset :12-148,
create_dataloaders :151-194). create_dataloaders yields the reference's dict batches
{clean_input_values, noisy_input_values, snr}; the mix, the validity checks and the
normalisation run on the GPU per batch (nrse_amd.data.MixedLoader), with the reference's retry
rules."""
import logging

import torch

from nrse_amd.data import (MAX_ATTEMPTS, GpuMixer, MixedLoader, MockPairs, SyntheticPairs,  # noqa: F401
                           WavPairs, create_dataloaders, create_raw_dataloaders, get_audio_files)

logger = logging.getLogger("nrse")


class NoiseRobustSpeechDataset(WavPairs):
    """The reference dataset (:13-148). Indexing returns the reference item
    {'clean_input_values' [1, L], 'noisy_input_values' [1, L], 'snr' int} (:140-144): the clean
    file and a random noise file are decoded / resampled / cropped on the host (audio_utils.py),
    and the SNR mix, peak and feature-extractor normalisation of the item run on the GPU of the
    calling process (nrse_snr_mix, the same kernel the batched loader uses). A failed mix
    re-draws the noise and SNR as the reference's `continue` does; after 5 attempts the item is
    None, as the reference's loop falls through to an implicit None. Batched training goes
    through create_dataloaders, which mixes whole batches at once."""

    def __init__(self, clean_data_path, noise_data_path, sample_rate=16000, max_audio_length=5.0,
                 snr_range=(0, 5, 10, 15, 20), feature_extractor=None):
        super().__init__(get_audio_files(clean_data_path), get_audio_files(noise_data_path), sample_rate,
                         max_audio_length, snr_range)
        self.feature_extractor = feature_extractor
        self._mixer = None
        print(f"Found {len(self.clean_files)} clean files and {len(self.noise_files)} noise files.")

    def _mix(self, raw):
        if self._mixer is None:
            norm = bool(getattr(self.feature_extractor, "do_normalize", True))
            self._mixer = GpuMixer(torch.device("cuda", torch.cuda.current_device()), norm)
        one = {"clean": raw["clean"][None], "noise": raw["noise"][None], "noise_len": raw["noise_len"][None],
               "snr": raw["snr"][None]}
        return self._mixer(one)

    def __getitem__(self, idx):
        try:
            raw = WavPairs.__getitem__(self, idx)
        except RuntimeError as e:
            logger.error(str(e))
            return None
        attempts = int(raw["attempts"])
        while True:
            out = self._mix(raw)
            if int(out["status"][0]) == 0:
                return {"clean_input_values": out["clean_input_values"][0].cpu(),
                        "noisy_input_values": out["noisy_input_values"][0].cpu(),
                        "snr": int(raw["snr"])}
            logger.warning(f"Noise addition failed, trying again (attempt {attempts})")
            if attempts >= MAX_ATTEMPTS:
                return None
            attempts += 1
            again = self.redraw(int(raw["index"]))
            if again is not None:
                raw = again
