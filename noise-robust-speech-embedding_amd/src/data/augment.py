"""Mirror of reference src/data/augment.py (add_noise_to_speech) on the fused GPU SNR-mix kernel."""
from nrse_amd.data import add_noise_to_speech  # noqa: F401
