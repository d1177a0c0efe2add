"""Synthetic MIND-shaped impressions and random-init weights.

There is no dataset or checkpoint in this environment, so the driver and the bench score
synthetic impressions of the reference's eval layout:

* history: ``hist_len ~ U{0..L}`` clicked-news rows, LEFT-padded to L with one fixed, nonzero pad
  news embedding (reader.py:101-110, :369); ``his_mask = position >= L - hist_len``
  (entities.py:395);
* candidates: C per impression (or ragged U[c_lo, c_hi]); labels with >= 1 click and >= 1
  non-click per impression (the reader keeps only such impressions, reader.py:374);
* embedding rows ~ N(0, 1)/sqrt(d).

Data is generated in blocks of ``BLOCK`` impressions, each from its own generator seeded by
(seed, block index): impression i's data depends only on (seed, i), never on how impressions are
sharded over ranks, so metrics are invariant to the world size.
"""
from __future__ import annotations

import dataclasses

import torch

BLOCK = 256


def _mix(seed: int, block: int) -> int:
    x = (seed * 0x9E3779B97F4A7C15 + block * 0xBF58476D1CE4E5B9 + 0x94D049BB133111EB) & (2**64 - 1)
    x ^= x >> 31
    x = (x * 0xD6E8FEB86659FD93) & (2**64 - 1)
    x ^= x >> 32
    return x & (2**63 - 1)


@dataclasses.dataclass
class Impressions:
    history: torch.Tensor        # [n, L, d]
    his_mask: torch.Tensor       # [n, L] bool
    candidates: torch.Tensor     # [n, C, d] dense, or [N, d] ragged
    cand_offsets: torch.Tensor | None  # [n+1] int32 (ragged) or None
    labels: torch.Tensor         # [n, C] or [N] int8
    impression_ids: torch.Tensor  # [n] int64 (global index)

    @property
    def n(self) -> int:
        return self.history.shape[0]

    @property
    def num_pairs(self) -> int:
        return self.labels.numel()


def pad_news(seed: int, d: int, device) -> torch.Tensor:
    g = torch.Generator(device=device).manual_seed(_mix(seed, 2**40))
    return torch.randn(d, generator=g, device=device) / d ** 0.5


def _block(seed, j, L, d, C, ragged, device, pad):
    g = torch.Generator(device=device).manual_seed(_mix(seed, j))
    n = BLOCK
    hist_len = torch.randint(0, L + 1, (n,), generator=g, device=device)
    E = torch.randn((n, L, d), generator=g, device=device) / d ** 0.5
    pos = torch.arange(L, device=device)
    mask = pos[None, :] >= (L - hist_len)[:, None]
    E = torch.where(mask[:, :, None], E, pad[None, None, :])
    if ragged:
        cnt = torch.randint(ragged[0], ragged[1] + 1, (n,), generator=g, device=device)
    else:
        cnt = torch.full((n,), C, device=device, dtype=torch.int64)
    N = int(cnt.sum())
    cand = torch.randn((N, d), generator=g, device=device) / d ** 0.5
    offs = torch.zeros(n + 1, dtype=torch.int64, device=device)
    offs[1:] = torch.cumsum(cnt, 0)
    lab = (torch.rand((N,), generator=g, device=device) < 0.2).to(torch.int8)
    pos_i = (torch.rand((n,), generator=g, device=device) * cnt).long().clamp_max(cnt - 1)
    neg_i = (pos_i + 1 + (torch.rand((n,), generator=g, device=device) * (cnt - 1)).long()) % cnt
    lab[offs[:-1] + pos_i] = 1
    lab[offs[:-1] + neg_i] = 0
    return E, mask, cand, cnt, lab


def impressions(seed: int, start: int, count: int, *, L: int, d: int, C: int = 40, ragged=None,
                device="cpu", dtype=torch.float32) -> Impressions:
    """Impressions [start, start+count) of the synthetic stream keyed by ``seed``."""
    device = torch.device(device)
    pad = pad_news(seed, d, device)
    j0, j1 = start // BLOCK, (start + count + BLOCK - 1) // BLOCK
    Es, Ms, Cs, Ns, Ls = [], [], [], [], []
    for j in range(j0, j1):
        E, M, cand, cnt, lab = _block(seed, j, L, d, C, ragged, device, pad)
        lo = max(start - j * BLOCK, 0)
        hi = min(start + count - j * BLOCK, BLOCK)
        cstart = int(cnt[:lo].sum())
        cend = cstart + int(cnt[lo:hi].sum())
        Es.append(E[lo:hi].to(dtype))
        Ms.append(M[lo:hi])
        Cs.append(cand[cstart:cend].to(dtype))
        Ns.append(cnt[lo:hi])
        Ls.append(lab[cstart:cend])
    hist = torch.cat(Es) if Es else torch.empty((0, L, d), device=device, dtype=dtype)
    mask = torch.cat(Ms) if Ms else torch.empty((0, L), device=device, dtype=torch.bool)
    cand = torch.cat(Cs) if Cs else torch.empty((0, d), device=device, dtype=dtype)
    cnt = torch.cat(Ns) if Ns else torch.empty((0,), device=device, dtype=torch.int64)
    lab = torch.cat(Ls) if Ls else torch.empty((0,), device=device, dtype=torch.int8)
    ids = torch.arange(start, start + count, device=device, dtype=torch.int64)
    if ragged:
        offs = torch.zeros(count + 1, dtype=torch.int32, device=device)
        offs[1:] = torch.cumsum(cnt, 0).to(torch.int32)
        return Impressions(hist, mask, cand, offs, lab, ids)
    return Impressions(hist, mask, cand.view(count, C, d), None, lab.view(count, C), ids)


def init_weights(seed: int, d: int, Dc: int, K: int, device="cpu"):
    """Random-init weights with the reference's initialisers (model.py:155-157, :198):
    W1 [Dc,d] and W2 [d,d] ~ nn.Linear default U(±1/sqrt(d)); Q [K,Dc] xavier_uniform(gain=5/3)."""
    g = torch.Generator(device="cpu").manual_seed(_mix(seed, 2**41))
    b = 1.0 / d ** 0.5
    W1 = (torch.rand((Dc, d), generator=g) * 2 - 1) * b
    W2 = (torch.rand((d, d), generator=g) * 2 - 1) * b
    gain = 5.0 / 3.0
    bq = gain * (6.0 / (Dc + K)) ** 0.5
    Q = (torch.rand((K, Dc), generator=g) * 2 - 1) * bq
    return W1.to(device), Q.to(device), W2.to(device)


@dataclasses.dataclass
class Behaviors:
    """Impressions as news ids (the reference's eval layout before the news encoder)."""
    his_ids: torch.Tensor        # [n, L] int32 rows of the news table (left pad = row 0, the pad news)
    his_mask: torch.Tensor       # [n, L] bool
    cand_ids: torch.Tensor       # [N] int32
    cand_offsets: torch.Tensor   # [n+1] int32
    labels: torch.Tensor         # [N] uint8
    impression_ids: torch.Tensor  # [n] int64

    @property
    def n(self) -> int:
        return self.his_ids.shape[0]


def news_table(seed: int, n_news: int, d: int, device="cpu", dtype=torch.float32) -> torch.Tensor:
    """[n_news, d] news embeddings ~ N(0,1)/sqrt(d); row 0 is the pad news (reader.py:101-110)."""
    g = torch.Generator(device="cpu").manual_seed(_mix(seed, 2**42))
    return (torch.randn((n_news, d), generator=g) / d ** 0.5).to(device=device, dtype=dtype)


def behaviors(seed: int, start: int, count: int, *, L: int, n_news: int, C=40, ragged=None,
              device="cpu") -> Behaviors:
    """Impressions [start, start+count): ids drawn per BLOCK of impressions from (seed, block), so
    any sharding sees the same data. ragged=(lo, hi) draws C_b ~ U[lo, hi]; >= 1 click and >= 1
    non-click per impression (reader.py:374)."""
    his, masks, cands, sizes, labs = [], [], [], [], []
    for j in range(start // BLOCK, (start + count + BLOCK - 1) // BLOCK):
        g = torch.Generator(device="cpu").manual_seed(_mix(seed ^ 0x5EED, j))
        n = BLOCK
        hl = torch.randint(0, L + 1, (n,), generator=g)
        ids = torch.randint(1, n_news, (n, L), generator=g)
        m = torch.arange(L)[None, :] >= (L - hl)[:, None]
        ids = torch.where(m, ids, torch.zeros_like(ids))
        cnt = torch.randint(ragged[0], ragged[1] + 1, (n,), generator=g) if ragged else torch.full((n,), C)
        N = int(cnt.sum())
        cid = torch.randint(1, n_news, (N,), generator=g)
        offs = torch.zeros(n + 1, dtype=torch.int64)
        offs[1:] = torch.cumsum(cnt, 0)
        lab = (torch.rand((N,), generator=g) < 0.2).to(torch.uint8)
        pos_i = (torch.rand((n,), generator=g) * cnt).long().clamp_max(cnt - 1)
        neg_i = (pos_i + 1 + (torch.rand((n,), generator=g) * (cnt - 1)).long()) % cnt
        lab[offs[:-1] + pos_i] = 1
        lab[offs[:-1] + neg_i] = 0
        lo, hi = max(start - j * BLOCK, 0), min(start + count - j * BLOCK, BLOCK)
        his.append(ids[lo:hi])
        masks.append(m[lo:hi])
        cands.append(cid[offs[lo]:offs[hi]])
        labs.append(lab[offs[lo]:offs[hi]])
        sizes.append(cnt[lo:hi])
    cnt = torch.cat(sizes) if sizes else torch.zeros(0, dtype=torch.int64)
    offs = torch.zeros(count + 1, dtype=torch.int32)
    offs[1:] = torch.cumsum(cnt, 0).to(torch.int32)
    dev = torch.device(device)
    return Behaviors(torch.cat(his).to(dev, torch.int32), torch.cat(masks).to(dev), torch.cat(cands).to(dev, torch.int32),
                     offs.to(dev), torch.cat(labs).to(dev), torch.arange(start, start + count, device=dev))


def fastformer_params(seed: int, device="cpu", affine_noise: bool = True) -> torch.Tensor:
    """Random FastFormer user-encoder parameters as the flat fp32 blob of miner_fastformer_pack
    (miner_amd.fastformer.PARAMS order). Weights ~ N(0, 0.02) as the reference's init
    (model.py:497-509); with ``affine_noise`` the biases ~ N(0, 0.05) and LayerNorm gains
    ~ 1 + N(0, 0.1) instead of the init's 0 / 1, so every parameter reaches the output."""
    from .fastformer import PARAMS
    g = torch.Generator(device="cpu").manual_seed(seed)
    parts = []
    for name, shape in PARAMS:
        if name.endswith("bias"):
            t = torch.randn(shape, generator=g) * 0.05 if affine_noise else torch.zeros(shape)
        elif "LayerNorm.weight" in name:
            t = 1.0 + torch.randn(shape, generator=g) * 0.1 if affine_noise else torch.ones(shape)
        else:
            t = torch.randn(shape, generator=g) * 0.02
        parts.append(t.reshape(-1))
    return torch.cat(parts).to(device)
