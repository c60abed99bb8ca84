"""Mirror of reference config/config_utils.py (load_config, parse_args, get_config)."""
from nrse_amd.config import apply_overrides, build_parser, get_config, load_config  # noqa: F401


def parse_args(argv=None):
    return build_parser().parse_args(argv)
