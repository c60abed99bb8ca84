"""Mirror of reference src/models/encoder.py (WavLMEncoder) on the MI355X path."""
from nrse_amd.model import WavLMEncoder  # noqa: F401
