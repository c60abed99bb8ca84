"""nrse_amd — MI355X-native (gfx950) BYOL-on-WavLM training path.

Host-side mirror of the reference's BYOL interface (src/models/byol.py, src/models/encoder.py,
src/data/augment.py, train_byol.py) over the hand-written HIP kernels of libnrse_hip.so.
"""
__version__ = "0.1.0"
