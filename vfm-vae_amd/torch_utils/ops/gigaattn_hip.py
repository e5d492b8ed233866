"""The decoder's self-attention with a learned null key / value (reference networks/utils/gigagan_utils.py
:53-91 SelfAttention.forward) as one autograd Function on the fp32 HIP kernels, laid out so that no
activation is copied between the products:

  forward   buf[b] = [null row ; (W_qkv x[b])^T]  -- token-major [P + 1, 3 h d]: the projection GEMM writes
            rows 1..P of a packed buffer whose row 0 holds (0, null_k, null_v), so q = buf[:, 1:, :hd],
            k = buf[:, :, hd:2hd], v = buf[:, :, 2hd:] are read in place by the attention kernels (the
            reference's torch.cat of the null key / value onto k / v is the buffer's row 0);
            o = attention(q, k, v) token-major [P, h d];  y[b] = W_out o[b]^T  ([C, P], channel-first)
  backward  dW_out = sum_b dy[b] o[b];  do[b] = (W_out^T dy[b])^T;  attention backward into ONE packed
            gradient buffer (dq rows 1..P, dk / dv rows 0..P);  d null = sum_b of row 0;
            dW_qkv = sum_b dbuf[b, 1:]^T x[b]^T;  dx[b] = W_qkv^T dbuf[b, 1:]^T

Every product is the fp32-equivalent f32x6 GEMM of gemm_hip (any operand strides), so the old path's
q .contiguous(), the two torch.cat copies, the output permute copy and the backward's view / stack copies
are gone. Same math as the unfused chain; the GEMMs see transposed operand orientations, so results
agree to fp32 rounding, not bit for bit (tests/test_decoder_attention_gpu.py)."""
import torch

from .. import custom_ops
from . import gemm_hip, kernel_timer
from .attn_hip import _lib, _s4


def _mm(A, B, **kw):
    """try_gemm (fp32-equivalent MFMA products) with the exact-fp32 torch product as the fallback for
    shapes / strides the kernels do not take."""
    out = gemm_hip.try_gemm(A, B, auto=True, **kw)
    if out is not None:
        return out
    red = kw.get('reduce_batch', False)
    r = torch.matmul(A, B)
    r = r.sum(0) if red else r
    if kw.get('out') is not None:
        kw['out'].copy_(r)
        return kw['out']
    return r


def _attn_fwd(q, k, v, scale):
    B, Nq, H, d = q.shape
    Nk = k.shape[1]
    o = torch.empty(B, Nq, H, d, dtype=torch.float32, device=q.device)
    lse = torch.empty(B, H, Nq, dtype=torch.float32, device=q.device)
    prec, _, tag = custom_ops.f32_precision()
    with kernel_timer.region(f"attention_fwd<{tag},{d}>", 4 * (2 * B * Nq * H * d + 2 * B * Nk * H * d),
                             4 * B * H * Nq * Nk * d, "mfma"):
        rc = _lib.vfm_attention_f32_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(),
                                        B, H, Nq, Nk, d, _s4(q), _s4(k), _s4(v), _s4(o), scale, prec,
                                        custom_ops.stream_ptr(q.device))
    custom_ops.check(rc, "vfm_attention_f32_fwd")
    return o, lse


class _NullKVSelfAttention(custom_ops.FastFunction):
    @staticmethod
    def forward(ctx, x3, wqkv, null_kv, wout, heads):
        B, C, P = x3.shape
        hd = wqkv.shape[0] // 3
        d = hd // heads
        buf = torch.empty(B, P + 1, 3 * hd, dtype=torch.float32, device=x3.device)
        buf[:, 0, :hd].zero_()
        buf[:, 0, hd:].copy_(null_kv.detach().reshape(1, 2 * hd).to(torch.float32))
        _mm(x3.transpose(1, 2), wqkv.detach().t(), out=buf[:, 1:, :], cache_b=True)   # rows 1..P: (W x)^T
        q = buf[:, 1:, :hd].view(B, P, heads, d)
        k = buf[:, :, hd:2 * hd].view(B, P + 1, heads, d)
        v = buf[:, :, 2 * hd:].view(B, P + 1, heads, d)
        o, lse = _attn_fwd(q, k, v, float(d) ** -0.5)
        y = _mm(wout.detach(), o.view(B, P, hd).transpose(1, 2), cache_a=True)        # [B, C, P]
        ctx.save_for_backward(x3, wqkv, wout, buf, o, lse)
        ctx.heads = heads
        ctx.dtypes = (wqkv.dtype, null_kv.dtype, wout.dtype)
        return y

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dy):
        x3, wqkv, wout, buf, o, lse = ctx.saved_tensors
        heads = ctx.heads
        B, C, P = x3.shape
        hd = wqkv.shape[0] // 3
        d = hd // heads
        dy = dy.contiguous()
        o2 = o.view(B, P, hd)
        dwout = _mm(dy, o2, out_dtype=torch.float32, reduce_batch=True) if ctx.needs_input_grad[3] else None
        do = _mm(dy.transpose(1, 2), wout.detach(), cache_b=True)                   # [B, P, hd] token-major
        dbuf = torch.empty_like(buf)
        dbuf[:, 0, :hd].zero_()
        dq = dbuf[:, 1:, :hd].view(B, P, heads, d)
        dk = dbuf[:, :, hd:2 * hd].view(B, P + 1, heads, d)
        dv = dbuf[:, :, 2 * hd:].view(B, P + 1, heads, d)
        q = buf[:, 1:, :hd].view(B, P, heads, d)
        k = buf[:, :, hd:2 * hd].view(B, P + 1, heads, d)
        v = buf[:, :, 2 * hd:].view(B, P + 1, heads, d)
        do4 = do.view(B, P, heads, d)
        delta = torch.empty(B, heads, P, dtype=torch.float32, device=dy.device)
        prec, _, tag = custom_ops.f32_precision()
        with kernel_timer.region(f"attention_bwd<{tag},{d}>", 4 * 4 * (B * P * heads * d + B * (P + 1) * heads * d),
                                 10 * B * heads * P * (P + 1) * d, "mfma"):
            rc = _lib.vfm_attention_f32_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), do4.data_ptr(),
                                            lse.data_ptr(), delta.data_ptr(), dq.data_ptr(), dk.data_ptr(),
                                            dv.data_ptr(), B, heads, P, P + 1, d, _s4(q), _s4(k), _s4(v), _s4(o),
                                            _s4(do4), _s4(dq), _s4(dk), _s4(dv), float(d) ** -0.5, prec,
                                            custom_ops.stream_ptr(dy.device))
        custom_ops.check(rc, "vfm_attention_f32_bwd")
        wdt, ndt, odt = ctx.dtypes
        dnull = dbuf[:, 0, hd:].sum(0).reshape(2, heads, d).to(ndt) if ctx.needs_input_grad[2] else None
        dqkv = dbuf[:, 1:, :]                                                      # [B, P, 3hd]
        dwqkv = _mm(dqkv.transpose(1, 2), x3.transpose(1, 2), out_dtype=torch.float32,
                    reduce_batch=True).to(wdt) if ctx.needs_input_grad[1] else None
        dx = _mm(wqkv.detach().t(), dqkv.transpose(1, 2), cache_a=True) if ctx.needs_input_grad[0] else None
        return dx, dwqkv, dnull, None if dwout is None else dwout.to(odt), None


def supported(x3, heads, dim_head):
    return (x3.is_cuda and x3.dtype == torch.float32 and dim_head == 64 and x3.shape[1] % 4 == 0
            and x3.shape[2] % 4 == 0 and (heads * dim_head) % 4 == 0)


def null_kv_self_attention(x3, wqkv, null_kv, wout, heads):
    """y [B, C, P] = W_out attention(q, [null_k; k], [null_v; v]) with (q, k, v) = W_qkv x3, x3 [B, C, P]
    fp32, wqkv [3 h d, C], null_kv [2, h, d], wout [C, h d]."""
    return _NullKVSelfAttention.apply(x3, wqkv, null_kv, wout, heads)
