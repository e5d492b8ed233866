"""Loader for the committed golden vectors (tests/golden/*.npz)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_cache = {}


def load(name):
    if name not in _cache:
        z = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
        arrays = {k: z[k] for k in z.files}
        meta = json.loads(str(arrays.pop("meta")))
        _cache[name] = (arrays, meta)
    return _cache[name]


def case(name, family, i):
    arrays, meta = load(name)
    prefix = f"{family}/{i}/"
    return {k[len(prefix):]: v for k, v in arrays.items() if k.startswith(prefix)}, meta[family][i]


def count(name, family):
    return len(load(name)[1][family])
