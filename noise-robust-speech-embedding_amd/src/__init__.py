"""Import-path mirror of the reference package layout (src.models / src.data / src.utils) over
nrse_amd: `from src.models.byol import BYOLSpeechModel, byol_loss` works unchanged."""
