"""Host-side training infrastructure (CPU): statistics collection semantics and the
shared setup helpers that train.py and bench.py both go through."""
import math

import pytest
import torch


def test_collector_intervals_and_keep_previous():
    from torch_utils import training_stats as ts
    a = ts.Collector(regex="T1/.*", keep_previous=True)
    b = ts.Collector(regex="T1/.*", keep_previous=False)
    ts.report("T1/x", [1.0, 3.0])
    a.update()
    b.update()
    assert a.num("T1/x") == 2 and a.mean("T1/x") == 2.0 and a.std("T1/x") == 1.0
    assert b.mean("T1/x") == 2.0
    a.update()                      # nothing new reported: a keeps the previous interval, b clears it
    b.update()
    assert a.mean("T1/x") == 2.0
    assert b.num("T1/x") == 0 and math.isnan(b.mean("T1/x"))
    ts.report("T1/x", 10.0)
    a.update()
    assert a.num("T1/x") == 1 and a.mean("T1/x") == 10.0 and a.std("T1/x") == 0.0
    assert a["T1/x"] == 10.0
    d = a.as_dict()
    assert d["T1/x"].num == 1
    with pytest.raises(KeyError):
        a.mean("Other/y")


def test_report_returns_value_and_ignores_empty():
    from torch_utils import training_stats as ts
    v = torch.ones(3)
    assert ts.report("T2/v", v) is v
    ts.report("T2/empty", [])
    c = ts.Collector(regex="T2/.*")
    assert c.num("T2/empty") == 0


def test_misc_helpers():
    from torch_utils import misc
    x = torch.zeros(2, 3, 4)
    misc.assert_shape(x, [2, None, 4])
    with pytest.raises(AssertionError):
        misc.assert_shape(x, [2, 4, 4])
    with pytest.raises(AssertionError):
        misc.assert_shape(x, [2, 3])
    a, b = torch.nn.BatchNorm1d(3), torch.nn.BatchNorm1d(3)
    with torch.no_grad():
        a.weight.fill_(2.0)
        a.running_mean.fill_(0.5)
    misc.copy_params_and_buffers(a, b, require_all=True)
    assert torch.equal(b.weight, a.weight) and torch.equal(b.running_mean, a.running_mean)
    assert len(misc.params_and_buffers(a)) == 5


def test_construct_iteration_matches_training_loop_setup(tmp_path):
    """bench.build and training_loop() share construct_networks / construct_iteration; on a GPU
    device the iteration replays the D-phase generator forward from graphs (the measured path)."""
    import json
    import net_cases
    from training.training_loop import construct_networks, construct_iteration, configure_backends
    vfm = tmp_path / net_cases.VFM_DIRNAME
    vfm.mkdir()
    json.dump(dict(net_cases.SIGLIP_CFG, layer_norm_eps=1e-6), open(vfm / "config.json", "w"))
    configure_backends(True)
    assert torch.backends.cuda.matmul.allow_tf32 is False
    dev = torch.device("cpu")
    G, G_ema, D = construct_networks(dict(net_cases.g_kwargs(str(vfm)), class_name="networks.generator.Generator"),
                                     dict(net_cases.D_KWARGS, class_name="networks.discriminator.ProjectedDiscriminator"),
                                     dev)
    opt = dict(class_name='torch.optim.Adam', lr=1e-3, betas=[0.0, 0.99], eps=1e-8)
    lk = dict(net_cases.loss_kwargs(str(vfm)), class_name="training.loss.TotalLoss")
    step = construct_iteration(G, D, G_ema, dev, lk, opt, opt, batch_size=2)
    assert getattr(step.loss, "graphed_nograd", None) is None       # CPU: eager
    assert step.G is G and step.G_ema is G_ema and step.D is D


@pytest.mark.parametrize("outcomes,hit", [(((1.0, 2, False), (0.5, 0, False)), True),     # both: unresized input
                                          (((1.0, 0, False), (0.5, 0, True)), False)])    # G phase resizes
def test_vfm_feature_reuse_is_exact(tmp_path, outcomes, hit):
    """The G phase reuses the D phase's frozen-tower features only when both phases feed the
    tower the same input, and the G-phase gradients equal a run that recomputes them."""
    import json
    import net_cases
    from det_init import det_init
    from networks.generator import Generator
    from networks.discriminator import ProjectedDiscriminator
    from training.loss import TotalLoss
    vfm = tmp_path / net_cases.VFM_DIRNAME
    vfm.mkdir()
    json.dump(dict(net_cases.SIGLIP_CFG, layer_norm_eps=1e-6), open(vfm / "config.json", "w"))
    grads = {}
    for reuse in (True, False):
        torch.manual_seed(0)
        G = Generator(label_dim=0, **net_cases.g_kwargs(str(vfm), use_equivariance_regularization=True,
                                                         img_resolution=128)).train().requires_grad_(False)
        D = ProjectedDiscriminator(c_dim=0, **net_cases.D_KWARGS).train().requires_grad_(False)
        det_init(G)
        det_init(D)
        loss = TotalLoss(device=torch.device('cpu'), G=G, D=D, **dict(net_cases.loss_kwargs(str(vfm)),
                                                                       use_equivariance_regularization=True))
        G.vfm_encoder.reuse_features = reuse
        img = torch.rand(2, 3, 128, 128, generator=torch.Generator().manual_seed(3))
        G.equivariance_transform.forced = outcomes[0]
        torch.manual_seed(1)
        loss.accumulate_gradients(phase='D', real_img=img, real_c=['x'] * 2, cur_nimg=0)
        G.equivariance_transform.forced = outcomes[1]
        for name, layer in G.named_modules():
            layer.requires_grad_(any(t in name for t in G.trainable_layers))
        torch.manual_seed(2)
        loss.accumulate_gradients(phase='G', real_img=img, real_c=['x'] * 2, cur_nimg=0)
        grads[reuse] = {n: p.grad.clone() for n, p in G.named_parameters() if p.grad is not None}
        if reuse:
            assert getattr(G.vfm_encoder, 'reuse_hits', 0) == (1 if hit else 0)
    assert grads[True].keys() == grads[False].keys() and grads[True]
    for n in grads[True]:
        assert torch.equal(grads[True][n], grads[False][n]), n


def test_kernel_timer_rocprof_names():
    """Timer regions map onto the kernel names rocprofv3 prints, so the bench's roofline
    average can be checked against the committed profile."""
    from torch_utils.ops import kernel_timer as kt
    assert kt.rocprof_name("gemm<f32x6,true,false,true>") == "gemm_kernel<true, false, 3, true, 8>"
    assert kt.rocprof_name("gemm<f32x3,true,false,true>") == "gemm_kernel<true, false, 2, true, 4>"
    assert kt.rocprof_name("gemm<bf16,false,true,false>[4x8x16x1]") == "gemm_kernel<false, true, 1, false, 4>"
    assert kt.rocprof_name("gemm8<f32x6,true,true,true>") == "gemm8_kernel<true, true, true, false, 0>"
    assert kt.rocprof_name("gemm8_gelu<2>") == "gemm8_kernel<true, false, false, false, 2>"
    assert kt.rocprof_name("gemm9_gelu<2>") == "gemm9p_kernel<true, false, false, 5>"
    assert kt.rocprof_name("gemm9<bf16,true,false,false>[64x64x64x1]").startswith("gemm9p_kernel<true, false, false, ")
    assert kt.rocprof_name("conv3x3_nhwc<f32x6,128>") == "conv3x3_kernel<256, 128, 3>"
    assert kt.rocprof_name("conv3x3_nhwc<f32x3,64>") == "conv3x3_kernel<128, 64, 2>"
    assert kt.rocprof_name("conv3x3_nhwc<f32x6,64>") == "conv3x3_kernel<128, 64, 3>"
    assert kt.rocprof_name("attention_fwd<f32x6,64>") == "attn32_fwd<3, 2>"
    assert kt.rocprof_name("attention_fwd<bf16,64>") == "attn_fwd_d64"
    assert kt.rocprof_name("dwconv2d_fwd<bf16,7>") == "dwr_fwd<__hip_bfloat16, 7>"
    assert kt.rocprof_name("gemm_ws<f32x6,true,true,true>") is None
    assert kt.rocprof_name("convnext_mlp_fwd<bf16,128,true>") == "mlp_fwd<128, true>"
    assert kt.rocprof_name("dwconv2d_mfma_bwd_weight<bf16,7>") == "dwm_bwd_w<7, "


def test_ema_copies_buffers_only_when_changed():
    """update_ema lerps the trainable parameters and copies a G buffer into G_ema only when
    the buffer changed since its last copy (reference training_loop.py:730-742 copies all)."""
    import copy
    from training.training_loop import TrainingIteration

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.lin = torch.nn.Linear(4, 4)
            self.register_buffer('const', torch.arange(4.0))
            self.trainable_layers = ['lin']

    G = Net()
    G_ema = copy.deepcopy(G)
    it = TrainingIteration.__new__(TrainingIteration)
    it.G, it.G_ema, it.batch_size, it.ema_kimg, it.ema_rampup, it._ema_pairs = G, G_ema, 4, 10.0, None, None
    with torch.no_grad():
        G.const.add_(1.0)
        G.lin.weight.add_(1.0)
    it.update_ema(1000)
    assert torch.equal(G_ema.const, G.const)
    v = G_ema.const._version
    it.update_ema(1000)                           # unchanged source: no copy
    assert G_ema.const._version == v
    with torch.no_grad():
        G.const.mul_(2.0)
    it.update_ema(1000)
    assert torch.equal(G_ema.const, G.const) and G_ema.const._version != v
    beta = 0.5 ** (4 / 10000.0)
    assert not torch.equal(G_ema.lin.weight, G.lin.weight)
    assert torch.isfinite(G_ema.lin.weight).all() and beta < 1


def test_ema_averages_frozen_tensor_that_comes_to_differ():
    """A frozen tensor equal in G and G_ema is left out of the lerp; once either side is written (a
    checkpoint loaded into G_ema) it is averaged again (version counters checked every step)."""
    import copy
    from training.training_loop import TrainingIteration

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.lin = torch.nn.Linear(4, 4)
            self.frozen = torch.nn.Linear(4, 4)
            self.trainable_layers = ['lin']

    G = Net()
    G_ema = copy.deepcopy(G)
    it = TrainingIteration.__new__(TrainingIteration)
    it.G, it.G_ema, it.batch_size, it.ema_kimg, it.ema_rampup, it._ema_pairs = G, G_ema, 4, 0.001, None, None
    it.update_ema(1000)
    assert torch.equal(G_ema.frozen.weight, G.frozen.weight)
    with torch.no_grad():
        G_ema.frozen.weight.zero_()                   # e.g. a checkpoint loaded into G_ema only
    it.update_ema(1000)                               # lerp weight 1 - beta = 1 - 0.5 ** (4 / 1)
    assert torch.allclose(G_ema.frozen.weight, (1 - 0.5 ** 4) * G.frozen.weight)


def test_graphed_forward_refused_without_opt_in(monkeypatch):
    """The HIP-graph replay of the D phase's generator forward is opt-in (torch reductions replay
    wrongly from HIP graphs): enabling it without VFM_EXPERIMENTAL_GRAPHS=1 raises."""
    import pytest
    from training.loss import TotalLoss
    monkeypatch.delenv("VFM_EXPERIMENTAL_GRAPHS", raising=False)
    obj = TotalLoss.__new__(TotalLoss)
    with pytest.raises(RuntimeError, match="experimental"):
        obj.enable_graphed_nograd_forward()
    obj.enable_graphed_nograd_forward(False)
    assert obj.graphed_nograd is None


def test_kernel_timer_sampling_is_unbiased():
    """region()'s launch sampling: exactly 1/every of each 2^16 launch indices, and every launch
    position of a region with 10 launches per step sampled (a plain stride of 4 or 16 would only
    ever time the even positions)."""
    from torch_utils.ops import kernel_timer as kt
    for every in (4, 16):
        kt._every = every
        hits = [c for c in range(1 << 16) if kt._sampled(c)]
        assert len(hits) == (1 << 16) // every
        assert {c % 10 for c in hits[:400]} == set(range(10))
    kt._every = 1


def test_fast_function_bypasses_apply_only_without_grad():
    """custom_ops.FastFunction: with grad mode off the forward runs directly (no graph node, the same
    values, a stand-in ctx whose saves are no-ops and whose needs_input_grad is all False); with grad
    mode on it is an ordinary autograd Function."""
    import torch
    from torch_utils import custom_ops

    seen = []

    class Twice(custom_ops.FastFunction):
        @staticmethod
        def forward(ctx, x, k):
            ctx.save_for_backward(x)
            ctx.k = k
            seen.append(ctx.needs_input_grad[0])
            # slicing as autograd's ctx allows (the paired VGG stack's forward: any(needs[:2]))
            assert len(ctx.needs_input_grad[:2]) == 2 and isinstance(any(ctx.needs_input_grad[:2]), bool)
            return x * k

        @staticmethod
        def backward(ctx, g):
            return g * ctx.k, None

    x = torch.arange(4.0, requires_grad=True)
    y = Twice.apply(x, 2.0)
    assert y.grad_fn is not None and seen[-1] is True
    y.sum().backward()
    assert torch.equal(x.grad, torch.full((4,), 2.0))
    with torch.no_grad():
        z = Twice.apply(x, 3.0)
    assert z.grad_fn is None and not z.requires_grad and seen[-1] is False
    assert torch.equal(z, torch.arange(4.0) * 3)


def test_kernel_timer_inactive_launches_are_counted_not_timed():
    """set_active(False): a region's launches keep being counted (the totals extrapolate from the timed
    launches to all of them) but none is timed; enable() re-activates."""
    from torch_utils.ops import kernel_timer as kt
    kt.enable(True, 1)
    kt.set_active(False)
    for _ in range(3):
        assert kt.region("x<f32>", 4) is kt._NULL
    assert kt._counts["x<f32>"] == 3
    kt.enable(False)
    kt.enable(True, 1)
    assert kt._active
    kt.enable(False)
