"""Vector quantisation of the discrete latent (multi-codebook, cosine/argmax lookup).

Same classes, buffers and parameter names as the reference
`networks/utils/quant_utils.py` (NormalizedEmbedding :33-49, VectorQuantizer
:58-133, VectorQuantizerM :136-199). The code lookup (normalise features and
codebook, argmax of the cosine, first index on ties) runs through
`torch_utils.ops.vq_ops.codebook_argmax`, which has a HIP kernel with a fixed
fp32 summation order so indices are reproducible bit-for-bit against the oracle.
"""
import torch
import torch.nn as nn
from torch.nn import functional as F

from torch_utils import distributed as dist
from torch_utils.ops import vq_ops


def get_entropy_loss(latent_embed, codebook_embed, inv_entropy_tau):
    d = latent_embed.square().sum(dim=1, keepdim=True) + codebook_embed.square().sum(dim=1)
    d = torch.addmm(d, latent_embed, codebook_embed.t(), alpha=-2, beta=1)
    logits = -d.float() * inv_entropy_tau
    prob, log_prob = logits.softmax(dim=-1), logits.log_softmax(dim=-1)
    per_sample_entropy = (-prob * log_prob).sum(dim=-1).mean()
    avg_prob = prob.mean(dim=0)
    codebook_entropy = (-avg_prob * torch.log(avg_prob + 1e-7)).sum()
    return per_sample_entropy - codebook_entropy


class NormalizedEmbedding(nn.Embedding):
    def __init__(self, num_embeddings, embedding_dim):
        super().__init__(num_embeddings=num_embeddings, embedding_dim=embedding_dim)

    def forward(self, idx):
        return F.embedding(idx, F.normalize(self.weight, dim=1), self.padding_idx, self.max_norm, self.norm_type,
                           self.scale_grad_by_freq, self.sparse)

    def get_norm_weight(self):
        return F.normalize(self.weight, dim=1)


class ResConv(nn.Conv2d):
    def __init__(self, embed_dim, quant_resi):
        ks = 3 if quant_resi < 0 else 1
        super().__init__(in_channels=embed_dim, out_channels=embed_dim, kernel_size=ks, stride=1, padding=ks // 2)
        self.resi_ratio = abs(quant_resi)

    def forward(self, h):
        return h.mul(1 - self.resi_ratio) + super().forward(h).mul_(self.resi_ratio)


class VectorQuantizer(nn.Module):
    def __init__(self, vocab_size, vocab_width, beta=0.25, use_entropy_loss=False, entropy_temp=0.01):
        super().__init__()
        self.beta = beta
        self.vocab_size = vocab_size
        self.vocab_width = vocab_width
        self.vocab_usage_record_times = 0
        self.register_buffer('vocab_usage', torch.zeros(self.vocab_size))
        self.codebook = NormalizedEmbedding(self.vocab_size, self.vocab_width)
        self.use_entropy_loss = use_entropy_loss
        self.inv_entropy_tau = 1 / entropy_temp

    def init_vocab(self, eini):
        if eini > 0:
            nn.init.trunc_normal_(self.codebook.weight.data, std=eini)
        elif eini < 0:
            base = self.vocab_width ** -0.5 / 36
            self.codebook.weight.data.uniform_(-abs(eini) * base, abs(eini) * base)

    def extra_repr(self):
        return f'beta={self.beta:g}'

    def forward(self, features):
        B, L, C = features.shape
        f = F.normalize(features.reshape(-1, C), dim=-1).float()
        codebook = self.codebook.get_norm_weight()
        indices = vq_ops.codebook_argmax(features.detach().reshape(-1, C).float(), self.codebook.weight.detach())
        entropy_loss = get_entropy_loss(f, codebook, self.inv_entropy_tau) if self.use_entropy_loss else 0
        f_hat = self.codebook(indices)
        vq_loss = F.mse_loss(f_hat.detach(), f).mul_(self.beta) + F.mse_loss(f_hat, f.detach())
        f_hat = (f_hat.detach() - f.detach()).add_(f)

        counts = indices.bincount(minlength=self.vocab_size).float()
        if self.training and dist.is_initialized():
            work = torch.distributed.all_reduce(counts, async_op=True)
            work.wait()
        counts /= counts.sum()
        vocab_usage = (counts > 0.01 / self.vocab_size).float().mean().mul_(100)
        if self.vocab_usage_record_times == 0:
            self.vocab_usage.copy_(counts)
        elif self.vocab_usage_record_times < 100:
            self.vocab_usage.mul_(0.9).add_(counts, alpha=0.1)
        else:
            self.vocab_usage.mul_(0.99).add_(counts, alpha=0.01)
        self.vocab_usage_record_times += 1
        return f_hat.view(B, L, C), vq_loss, entropy_loss, vocab_usage

    def f_to_idx(self, features):
        B, L, C = features.shape
        idx = vq_ops.codebook_argmax(features.detach().reshape(-1, C).float(), self.codebook.weight.detach())
        return idx.view(B, L)


class VectorQuantizerM(nn.Module):
    """`num_codebooks` independent quantisers over equal chunks of the feature width."""

    def __init__(self, vocab_size, vocab_width, beta=0.25, use_entropy_loss=False, entropy_temp=0.01,
                 num_codebooks=16):
        super().__init__()
        self.num_codebooks = num_codebooks
        self.codebooks = nn.ModuleList([
            VectorQuantizer(vocab_size=vocab_size // num_codebooks, vocab_width=vocab_width // num_codebooks,
                            beta=beta, use_entropy_loss=use_entropy_loss, entropy_temp=entropy_temp)
            for _ in range(num_codebooks)])

    def init_vocab(self, eini):
        for cb in self.codebooks:
            cb.init_vocab(eini)

    def f_to_idx(self, features):
        chunk = features.shape[-1] // self.num_codebooks
        parts = features.split(chunk, dim=-1)
        return torch.stack([cb.f_to_idx(p) for cb, p in zip(self.codebooks, parts)], dim=1)

    def idx_to_f(self, indices):
        assert indices.shape[1] == self.num_codebooks
        feats = [cb.codebook(indices[:, i].flatten(start_dim=1)) for i, cb in enumerate(self.codebooks)]
        return torch.cat(feats, dim=-1)

    def forward(self, features):
        chunk = features.shape[-1] // self.num_codebooks
        parts = features.split(chunk, dim=-1)
        outs, vq, ent, usage = [], 0., 0., 0.
        for cb, p in zip(self.codebooks, parts):
            f_hat, l_vq, l_ent, u = cb(p)
            outs.append(f_hat)
            vq += l_vq
            ent += l_ent
            usage += u
        n = self.num_codebooks
        return torch.cat(outs, dim=-1), vq / n, ent / n, usage / n
