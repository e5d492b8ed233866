"""Config plumbing used by the YAML surface.

Mirrors the parts of the reference `dnnlib/util.py` that the training path and
the tools touch: `EasyDict` (`dnnlib/util.py:39`), `get_obj_by_name` /
`construct_class_by_name` / `call_func_by_name` (`dnnlib/util.py:250-310`) and a
tee-style `Logger` (`dnnlib/util.py:60-120`).
"""
import importlib
import os
import sys
import tempfile
from typing import Any


class EasyDict(dict):
    """dict with attribute access."""

    def __getattr__(self, name: str) -> Any:
        try:
            return self[name]
        except KeyError:
            raise AttributeError(name)

    def __setattr__(self, name: str, value: Any) -> None:
        self[name] = value

    def __delattr__(self, name: str) -> None:
        del self[name]


class Logger:
    """Duplicates stdout/stderr into a log file (reference `dnnlib.util.Logger`)."""

    def __init__(self, file_name=None, file_mode="w", should_flush=True):
        self.file = open(file_name, file_mode) if file_name is not None else None
        self.should_flush = should_flush
        self.stdout = sys.stdout
        self.stderr = sys.stderr
        sys.stdout = self
        sys.stderr = self

    def write(self, text):
        if isinstance(text, bytes):
            text = text.decode()
        if not text:
            return
        if self.file is not None:
            self.file.write(text)
        self.stdout.write(text)
        if self.should_flush:
            self.flush()

    def flush(self):
        if self.file is not None:
            self.file.flush()
        self.stdout.flush()

    def close(self):
        self.flush()
        if sys.stdout is self:
            sys.stdout = self.stdout
        if sys.stderr is self:
            sys.stderr = self.stderr
        if self.file is not None:
            self.file.close()
            self.file = None


def make_cache_dir_path(*paths: str) -> str:
    base = os.environ.get("DNNLIB_CACHE_DIR") or os.path.join(tempfile.gettempdir(), "dnnlib")
    return os.path.join(base, *paths)


def get_module_from_obj_name(obj_name: str):
    """Split 'a.b.c.Name' into (module, 'Name'), trying the longest importable prefix."""
    parts = obj_name.split(".")
    for i in range(len(parts) - 1, 0, -1):
        mod_name = ".".join(parts[:i])
        try:
            module = importlib.import_module(mod_name)
        except ModuleNotFoundError as e:
            if e.name is not None and not mod_name.startswith(e.name):
                raise
            continue
        return module, ".".join(parts[i:])
    return importlib.import_module(obj_name), ""


def get_obj_by_name(name: str) -> Any:
    module, local = get_module_from_obj_name(name)
    obj = module
    for attr in local.split(".") if local else []:
        obj = getattr(obj, attr)
    return obj


def call_func_by_name(*args, func_name: str = None, **kwargs) -> Any:
    assert func_name is not None
    fn = get_obj_by_name(func_name)
    assert callable(fn)
    return fn(*args, **kwargs)


def construct_class_by_name(*args, class_name: str = None, **kwargs) -> Any:
    return call_func_by_name(*args, func_name=class_name, **kwargs)


def get_top_level_function_name(obj: Any) -> str:
    return obj.__module__ + "." + obj.__name__
