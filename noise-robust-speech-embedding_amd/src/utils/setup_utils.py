"""Mirror of reference src/utils/setup_utils.py (set_seed)."""
import numpy as np
import torch


def set_seed(seed=42):
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    np.random.seed(seed)
