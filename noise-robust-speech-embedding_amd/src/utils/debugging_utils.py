"""Drop-in for the reference src/utils/debugging_utils.py (check_audio_tensor, :4-30): the four
reductions run as one nrse_health kernel; decisions and messages follow the reference."""
from nrse_amd.health import check_audio_tensor  # noqa: F401
