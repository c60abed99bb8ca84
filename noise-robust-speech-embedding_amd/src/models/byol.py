"""Mirror of reference src/models/byol.py (BYOLSpeechModel, byol_loss) on the MI355X path."""
from nrse_amd.model import BYOLSpeechModel, byol_loss  # noqa: F401
