"""torch_utils/ops/kernel_timer.py host logic (no GPU): the target mode bench.py runs its timed steps in (only the
dominant region counted and sampled, every other region a no-op), the dominant-region pick and the merge of the
pre-pass ranking into the roofline object."""
from torch_utils.ops import kernel_timer as kt


def test_target_mode_bypasses_other_regions():
    kt._enable(True, 20)
    try:
        kt.set_target("gemm9<f32x6,true,false,true>")
        assert kt.region("group_norm_bwd<bf16>", 10) is kt._NULL
        assert "group_norm_bwd<bf16>" not in kt._counts
        kt.set_active(False)                       # counted, not timed (no native events on the CPU)
        assert kt.region("gemm9<f32x6,true,false,true>", 10, 5.0, "mfma") is kt._NULL
        assert kt._counts == {"gemm9<f32x6,true,false,true>": 1}
        kt._enable(True, 20)                       # enable() clears the target
        assert kt._target is None
        kt.set_active(False)
        kt.region("group_norm_bwd<bf16>", 10)
        assert kt._counts == {"group_norm_bwd<bf16>": 1}
    finally:
        kt._enable(False)


def test_dominant_name_and_prepass_merge(monkeypatch):
    pre = {"a<bf16>": dict(launches=10, timed_launches=1, total_ms=5.0, bytes=1e9, flops=0.0, flops_all=0.0, bound="hbm"),
           "gemm9<bf16,true,true,false>": dict(launches=20, timed_launches=2, total_ms=9.0, bytes=1e9, flops=4e12,
                                               flops_all=4e12, bound="mfma"),
           "vendor_gemm<f32,x>": dict(launches=5, timed_launches=1, total_ms=50.0, bytes=1e9, flops=1e12,
                                      flops_all=1e12, bound="mfma")}
    assert kt.dominant_name(pre) == "gemm9<bf16,true,true,false>"     # library GEMMs never lead
    timed = {"gemm9<bf16,true,true,false>": dict(launches=40, timed_launches=2, total_ms=20.0, bytes=2e9, flops=8e12,
                                                 flops_all=8e12, bound="mfma")}
    monkeypatch.setattr(kt, "summary", lambda: dict(timed))
    roof = kt.dominant_roofline(8000.0, 2500.0, prepass=(pre, 2.0))
    assert roof["kernel"] == "gemm9<bf16,true,true,false>"
    assert roof["launches"] == 40 and roof["ms_total"] == 20.0            # the timed steps' own record
    assert roof["all_kernels"]["a<bf16>"]["ms"] == 10.0                   # pre-pass totals scaled x2
    assert roof["all_kernels"]["a<bf16>"]["launches"] == 20
    assert roof["vendor_top"]["kernel"] == "vendor_gemm<f32,x>"
