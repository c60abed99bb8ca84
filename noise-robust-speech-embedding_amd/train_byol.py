"""Drop-in for the reference `python train_byol.py --config <yaml> [--device ...]` entry point."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from nrse_amd.train import EarlyStopping, main, train_one_epoch, validate_model  # noqa: E402,F401

if __name__ == "__main__":
    main()
