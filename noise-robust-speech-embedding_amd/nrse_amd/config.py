"""YAML + CLI configuration, same schema and overrides as the reference
(config/config_utils.py:21-65; config/default_wavlm-large_byol.yaml:1-59)."""
from __future__ import annotations

import argparse
from typing import Any, Dict

import yaml


def load_config(config_path: str) -> Dict[str, Any]:
    with open(config_path, "r") as f:
        return yaml.safe_load(f)


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="NRSE: Noise Robust Speech Embeddings (MI355X)")
    p.add_argument("--config", type=str, default="config/default.yaml", help="Path to configuration file")
    p.add_argument("--device", type=str, default=None, help="Device to use (cuda[:i])")
    p.add_argument("--batch_size", type=int, default=None, help="Batch size for training (per GPU)")
    p.add_argument("--epochs", type=int, default=None, help="Number of training epochs")
    p.add_argument("--lr", type=float, default=None, help="Learning rate")
    p.add_argument("--task", type=str, default="both", choices=["categorical", "dimensional", "both"],
                   help="Which emotion recognition task to train (parsed, unused by BYOL training)")
    # MI355X additions (defaults keep the reference behaviour)
    p.add_argument("--dtype", type=str, default="bf16", choices=["bf16", "bf16sw", "f32"],
                   help="compute dtype of GEMM/attention operands (f32 = exact parity mode; bf16sw = bf16 "
                        "activations x split hi+lo bf16 weights in the forward, the north-star 1e-3 mode)")
    p.add_argument("--max_steps", type=int, default=None, help="stop after this many optimizer steps")
    p.add_argument("--mock_items", type=int, default=None,
                   help="train on test/create_mock_dataset.py-style mock pairs (configs[0] plumbing)")
    p.add_argument("--sync_bn", action="store_true", help="DDP: SyncBatchNorm in the heads")
    p.add_argument("--bf16_allreduce", action="store_true", help="DDP: gradient all-reduce in bf16 on the wire")
    return p


def apply_overrides(config: Dict[str, Any], args) -> Dict[str, Any]:
    """CLI arguments override YAML values (config_utils.py:49-65)."""
    import torch
    if args.device is not None:
        config["device"] = args.device
    else:
        config["device"] = "cuda" if torch.cuda.is_available() else "cpu"
    if args.batch_size is not None:
        config["training"]["batch_size"] = args.batch_size
    if args.epochs is not None:
        config["training"]["num_epochs"] = args.epochs
    if args.lr is not None:
        config["training"]["learning_rate"] = args.lr
    config.setdefault("runtime", {})
    config["runtime"]["dtype"] = getattr(args, "dtype", "bf16")
    config["runtime"]["max_steps"] = getattr(args, "max_steps", None)
    config["runtime"]["sync_bn"] = bool(getattr(args, "sync_bn", False))
    config["runtime"]["bf16_allreduce"] = bool(getattr(args, "bf16_allreduce", False))
    if getattr(args, "mock_items", None):
        config["data"]["mock_items"] = args.mock_items
    return config


def get_config(argv=None) -> Dict[str, Any]:
    args = build_parser().parse_args(argv)
    return apply_overrides(load_config(args.config), args)
