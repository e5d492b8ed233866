"""Minimal config/utility namespace mirroring the reference's `dnnlib` surface
(`dnnlib/util.py`: EasyDict, construct_class_by_name, Logger) used by train.py,
the training loop and the YAML configs."""
from .util import EasyDict, make_cache_dir_path  # noqa: F401
