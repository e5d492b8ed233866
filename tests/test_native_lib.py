"""The C-ABI library loads and exports every symbol include/*.h declares.
No compute calls (there is no GPU in the build container)."""
import ctypes
import glob
import os
import re

from conftest import ROOT

LIB = os.path.join(ROOT, "vfm-vae_amd", "lib", "libvfmvae_hip.so")


def declared_symbols():
    syms = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        syms.update(re.findall(r"\b(vfm_\w+)\s*\(", src))
    return sorted(syms)


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "vfm_upfirdn2d" in syms and "vfm_bias_act" in syms and "vfm_filtered_lrelu" in syms
    assert len(syms) >= 5


def test_library_exports_all_declared_symbols():
    assert os.path.exists(LIB), "run __graft_entry__.build() first"
    lib = ctypes.CDLL(LIB)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_version_string():
    lib = ctypes.CDLL(LIB)
    lib.vfm_version.restype = ctypes.c_char_p
    assert b"gfx950" in lib.vfm_version()


def test_python_signatures_cover_header():
    import torch_utils.custom_ops as co
    declared = set(declared_symbols()) - {"vfm_version"}
    assert declared == set(co.SIGNATURES), declared ^ set(co.SIGNATURES)


def test_argument_validation_without_gpu():
    """Invalid arguments are rejected before any device work (VFM_ERR_ARGS = -2)."""
    import torch_utils.custom_ops as co
    lib = co.get_native()
    xs = (ctypes.c_longlong * 4)(1, 1, 1, 1)
    rc = lib.vfm_upfirdn2d(None, None, None, 0, 1, 1, 1, 1, xs, 1, 1, xs, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 1.0, None)
    assert rc == -2
    rc = lib.vfm_bias_act(None, None, None, None, None, None, 0, 4, 0, 1, 0.0, 1.0, -1.0, 1, 1, None)
    assert rc == -2
    # unsupported up factor -> "no kernel" (-1), the reference's fallback signal
    p = ctypes.c_void_p(16)
    rc = lib.vfm_filtered_lrelu(p, p, p, None, None, p, 0, 1, 1, 4, 4, xs, 4, 4, xs, 1, 1, 1, 1, 3, 1, 0, 0,
                                0, 0, 0, 0, 0, 1.0, 0.2, float("inf"), 0, None)
    assert rc == -1


def test_dwconv_partial_tiles_host_query():
    """vfm_dwconv2d_bwd_weight_tiles is pure host logic: the number of partial slices the
    weight-gradient kernel writes per channel (row-streaming path: waves per channel; tile path:
    column tiles x batch)."""
    import torch_utils.custom_ops as co
    lib = co.get_native()
    assert lib.vfm_dwconv2d_bwd_weight_tiles(2, 8, 256, 256, 7, 3) == 64    # 2 samples x 32 bands of 8 rows
    assert lib.vfm_dwconv2d_bwd_weight_tiles(2, 8, 16, 16, 3, 1) == 1       # 16 units per wave
    assert lib.vfm_dwconv2d_bwd_weight_tiles(3, 2, 5, 130, 3, 1) == 9       # 3 column tiles x 3 samples
    assert lib.vfm_dwconv2d_bwd_weight_tiles(1, 1, 5, 130, 3, 1) == 3
    assert lib.vfm_dwconv2d_bwd_weight_tiles(1, 1, 2, 2, 7, 0) == -2      # empty output -> VFM_ERR_ARGS


def test_torch_library_schemas():
    """TORCH_LIBRARY(vfmvae) registers the reference plugins' ops with their schemas
    (reference upfirdn2d.cpp:16, bias_act.cpp:32, filtered_lrelu.cpp:16,213), backed by the
    extern "C" launchers; argument checks run before any device work."""
    import pytest
    import torch
    import torch_utils.custom_ops as co
    ops = co.get_torch_ops()
    sch = {n: str(getattr(ops, n).default._schema) for n in ("upfirdn2d", "bias_act", "filtered_lrelu",
                                                                "filtered_lrelu_act_")}
    assert sch["upfirdn2d"] == ("vfmvae::upfirdn2d(Tensor x, Tensor f, int upx, int upy, int downx, int downy, "
                                "int padx0, int padx1, int pady0, int pady1, bool flip, float gain) -> Tensor")
    assert sch["bias_act"] == ("vfmvae::bias_act(Tensor x, Tensor b, Tensor xref, Tensor yref, Tensor dy, int grad, "
                               "int dim, int act, float alpha, float gain, float clamp) -> Tensor")
    assert sch["filtered_lrelu"].endswith("bool flip_filters, bool writeSigns) -> (Tensor, Tensor, int)")
    assert sch["filtered_lrelu_act_"].startswith("vfmvae::filtered_lrelu_act_(Tensor(a!) x, Tensor si")
    # CPU tensors: the ops are registered for the CUDA (ROCm) dispatch key only
    with pytest.raises(NotImplementedError):
        ops.upfirdn2d(torch.zeros(1, 1, 4, 4), torch.ones(1, 1), 1, 1, 1, 1, 0, 0, 0, 0, False, 1.0)


def test_torch_ops_load_first_in_fresh_process():
    """get_torch_ops() as the first native call of a process (what smoke() does through upfirdn2d)
    returns: it takes the loader lock and loads the kernel library under it (a non-reentrant lock
    deadlocked there)."""
    import subprocess
    import sys
    root = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r); from torch_utils import custom_ops; "
            "print(custom_ops.get_torch_ops() is not None)" % (root + "/vfm-vae_amd"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("True"), r.stderr[-2000:]
