"""Import-path mirror of the reference `config` package: `from config.config_utils import
get_config` works unchanged (reference config/config_utils.py:21-65)."""
