"""The fused Adam + G_ema step (csrc/adam.hip via training_loop.fast_adam_step / torch_utils/ops/adam_hip.py)
against torch.optim.Adam(fused=True).step() followed by torch._foreach_lerp_ (the reference's opt.step() and
G_ema update, training/training_loop.py:722-742) on twin parameter sets on cuda:0: vectorised and ragged
tensors (n % 4 != 0), gradients as unaligned views of one flat buffer (the FlatGradSync layout), weight decay,
a parameter without a gradient on one step, several steps. Tolerance: the kernel mirrors the fused kernel's
expression forms and precisions, so the parameters, moments and EMA copies agree to 2 ulp-scale relative
error (2e-6 of max |value|) after every step; the step counters exactly."""
import pytest
import torch

import dnnlib
from training.training_loop import fast_adam_step

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _params(seed):
    g = torch.Generator().manual_seed(seed)
    shapes = [(64, 33), (257,), (1024, 16), (3,), (8192 * 2 + 5,)]
    return [torch.nn.Parameter(torch.randn(s, generator=g).to(DEV)) for s in shapes]


def _rel(a, b):
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


@pytest.mark.parametrize("wd", [0.0, 0.01])
def test_fused_adam_ema_matches_torch(wd):
    pa, pb = _params(0), _params(0)
    ema_a = [p.detach().clone() * 0.9 for p in pa]
    ema_b = [e.clone() for e in ema_a]
    kw = dict(lr=2e-3, betas=(0.5, 0.99), eps=1e-8, weight_decay=wd, fused=True)
    oa, ob = torch.optim.Adam(pa, **kw), torch.optim.Adam(pb, **kw)
    phase = dnnlib.EasyDict(opt=ob)
    # gradients of b live in one flat buffer at odd offsets (unaligned views), as FlatGradSync lays them out
    n = sum(p.numel() for p in pb) + 7
    flat = torch.zeros(n, device=DEV)
    offs, o = [], 3
    for p in pb:
        offs.append(o)
        o += p.numel()
    pairs = {id(p): e for p, e in zip(pb, ema_b)}
    g = torch.Generator().manual_seed(5)
    fast_steps = 0
    for it in range(5):
        w = 1.0 - 0.5 ** (it + 1) / 4
        grads = [torch.randn(p.shape, generator=g).to(DEV) for p in pa]
        drop = 1 if it == 3 else None
        for i, (p, q, gr) in enumerate(zip(pa, pb, grads)):
            if i == drop:
                p.grad = q.grad = None
                continue
            p.grad = gr.clone()
            view = flat[offs[i]:offs[i] + q.numel()].view(q.shape)
            view.copy_(gr)
            q.grad = view
        oa.step()
        done = fast_adam_step(phase, (pairs, w))
        if done is False:
            ob.step()
            done = set()
        else:
            fast_steps += 1
        # the reference's EMA over every pair, for a; for b the pairs the fused step did not cover
        torch._foreach_lerp_(ema_a, [p.detach() for p in pa], w)
        rest = [(e, p) for p, e in zip(pb, ema_b) if id(p) not in done]
        if rest:
            torch._foreach_lerp_([e for e, _ in rest], [p.detach() for _, p in rest], w)
        torch.cuda.synchronize()
        for p, q, ea, eb in zip(pa, pb, ema_a, ema_b):
            assert _rel(q.detach(), p.detach()) <= 2e-6, (it, p.shape)
            assert _rel(eb, ea) <= 2e-6, (it, p.shape)
            sa, sb = oa.state[p], ob.state[q]
            if sa:
                assert _rel(sb["exp_avg"], sa["exp_avg"]) <= 2e-6
                assert _rel(sb["exp_avg_sq"], sa["exp_avg_sq"]) <= 2e-6
                assert float(sb["step"]) == float(sa["step"])
    # step 0 creates the state (regular path); step 3 rebuilds without the dropped parameter; at step 4 the step
    # counters differ (that parameter missed one), so the rebuilt list runs torch's fused Adam
    assert fast_steps == 4


def test_fused_adam_hip_is_used():
    """The fused step runs the native kernel (not torch's fused Adam) on ROCm."""
    from torch.utils._python_dispatch import TorchDispatchMode
    p = [torch.nn.Parameter(torch.randn(100, device=DEV))]
    opt = torch.optim.Adam(p, lr=1e-3, fused=True)
    phase = dnnlib.EasyDict(opt=opt)
    for _ in range(2):
        p[0].grad = torch.randn(100, device=DEV)
        if fast_adam_step(phase) is False:
            opt.step()

    class Rec(TorchDispatchMode):
        names = []

        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            Rec.names.append(str(func))
            return func(*args, **(kwargs or {}))

    p[0].grad = torch.randn(100, device=DEV)
    with Rec():
        assert fast_adam_step(phase) is not False
    assert not any("fused_adam" in n for n in Rec.names), Rec.names


def test_direct_mode_grads_match_flat_buffer():
    """FlatGradSync direct mode (world size 1 on a GPU: autograd's own gradient tensors, the gain and nan_to_num
    applied inside the Adam kernel, csrc/adam.hip vfm_adam_ema_step_raw) against the flat-buffer mode (gather,
    flat *= gain, nan_to_num over the buffer, reference training_loop.py:281-289) on twin modules: two microbatches
    per step, gain 2, non-finite gradient entries, a parameter without a gradient on one step, the G_ema lerp;
    bit-identical parameters, moments and EMA copies after every step."""
    from training import training_loop as tl

    def make():
        torch.manual_seed(0)
        return torch.nn.Sequential(torch.nn.Linear(33, 64), torch.nn.GELU(), torch.nn.Linear(64, 5),
                                   torch.nn.Linear(5, 7)).to(DEV)

    mods = [make(), make()]
    phases, emas = [], []
    for direct, m in zip((True, False), mods):
        old = tl.DIRECT_GRADS
        tl.DIRECT_GRADS = direct
        try:
            sync = tl.FlatGradSync(m, collective=False)
            m.requires_grad_(True)
            sync.prepare()
        finally:
            tl.DIRECT_GRADS = old
        assert sync.direct == direct
        opt = torch.optim.Adam(m.parameters(), lr=1e-2, betas=(0.5, 0.99), eps=1e-8, fused=True)
        phases.append(dnnlib.EasyDict(opt=opt, sync=sync))
        emas.append([p.detach().clone() for p in m.parameters()])
    g = torch.Generator().manual_seed(3)
    hip_steps = [0, 0]
    # step 0 creates the state (regular opt.step), 1-4 run the native kernel (2: +-inf, 3: nan gradient entries,
    # 4: the last layer without a gradient), 5 torch's fused Adam (the step counters differ since step 4)
    for it in range(6):
        xs = [torch.randn(16, 33, generator=g).to(DEV) for _ in range(2)]
        for k, (m, phase, ema) in enumerate(zip(mods, phases, emas)):
            phase.sync.prepare()
            for mb, x in enumerate(xs):
                y = m[:3](x) if it == 4 else m(x)
                loss = (y ** 2).sum()
                if it == 2 and mb == 1:
                    loss = loss + m[0].bias[0] * float("inf") - m[0].bias[1] * float("inf")
                if it == 3 and mb == 0:
                    loss = loss + m[2].weight[0, 0] * float("nan")
                loss.backward()
            phase.sync.finish(gain=2)
            pairs = {id(p): e for p, e in zip(m.parameters(), ema)}
            done = tl.fast_adam_step(phase, (pairs, 0.25))
            if done is False:
                phase.opt.step()
                done = set()
            hip_steps[k] += bool(done)
            rest = [(e, p) for p, e in zip(m.parameters(), ema) if id(p) not in done and p.grad is not None]
            if rest:
                torch._foreach_lerp_([e for e, _ in rest], [p.detach() for _, p in rest], 0.25)
            phase.opt.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        for (na, pa), (_, pb), ea, eb in zip(mods[0].named_parameters(), mods[1].named_parameters(), *emas):
            assert torch.isfinite(pa).all(), (it, na)
            assert torch.equal(pa, pb), (it, na)
            assert torch.equal(ea, eb), (it, na)
            sa, sb = phases[0].opt.state[pa], phases[1].opt.state[pb]
            assert torch.equal(sa["exp_avg"], sb["exp_avg"]) and torch.equal(sa["exp_avg_sq"], sb["exp_avg_sq"])
    assert phases[0].sync.raw is None
    assert hip_steps == [4, 4]
