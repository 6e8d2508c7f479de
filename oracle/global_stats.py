"""CPU restatement of the data-parallel decomposition of the batch-coupled losses (SURVEY.md §8e
option ii): ContrastRegionLoss (modules/trainer.py:89-130) and ContrastEdgeLoss
(modules/trainer.py:133-184) computed from per-shard partial sums that are added over ranks.

TEST INFRASTRUCTURE ONLY (the checker, never the product path).  Mirrors the phase kernels of
ducosy-gan_amd/csrc/loss.hip (dcs_loss_contrast_region_partial/_finish and
dcs_loss_contrast_edge_partial/_hist/_select/_topk/_finish): the same quantities, float64
sums, and the same radix select of the k-th largest edge magnitude over summed 256-bin
histograms of the float32 bit patterns.  Pinned against oracle/ref_torch.py's whole-batch
contrast_region_loss / contrast_edge_loss in tests/test_cpu_global_stats.py.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .ref_torch import edges


# ---------------------------------------------------------------------------------------
# ContrastRegionLoss: red = {sum m|pp - tp|, sum p, sum p^2, sum t, sum t^2, n, nq}
# ---------------------------------------------------------------------------------------
def region_partial(pred, target, source, threshold):
    """modules/trainer.py:114-128 split into sums: the region term's numerator and the
    moments of pred / target over this shard."""
    pp, tp, sp = F.avg_pool2d(pred, 8, 8), F.avg_pool2d(target, 8, 8), F.avg_pool2d(source, 8, 8)
    m = torch.sigmoid(5.0 * ((tp - sp) - threshold))
    p, t = pred.double(), target.double()
    return torch.stack([(m * (pp - tp).abs()).double().sum(), p.sum(), (p * p).sum(), t.sum(), (t * t).sum(),
                        torch.tensor(float(pred.numel()), dtype=torch.float64),
                        torch.tensor(float(pp.numel()), dtype=torch.float64)])


def _mean_std(s1, s2, n):
    """mean and unbiased std (torch.std default) from a sum and a sum of squares."""
    mean = s1 / n
    return mean, torch.sqrt(torch.clamp((s2 - n * mean * mean) / (n - 1), min=0.0))


def region_finish(red, weight):
    """weight * (region + 0.5 * (|mean p - mean t| + |std p - std t|)) of the whole batch."""
    mp, sp = _mean_std(red[1], red[2], red[5])
    mt, st = _mean_std(red[3], red[4], red[5])
    return weight * (red[0] / red[6] + 0.5 * ((mp - mt).abs() + (sp - st).abs()))


# ---------------------------------------------------------------------------------------
# ContrastEdgeLoss: red = {sum ep, sum ep^2, sum et, sum et^2, n, sum ep>tp, #ep==tp, sum et>tt, #et==tt}
# ---------------------------------------------------------------------------------------
def edge_partial(pred, target):
    """Sobel magnitudes of this shard (kept for the later phases) and their moments."""
    pe, te = edges(pred).flatten(), edges(target).flatten()
    a, b = pe.double(), te.double()
    red = torch.zeros(9, dtype=torch.float64)
    red[:5] = torch.stack([a.sum(), (a * a).sum(), b.sum(), (b * b).sum(),
                           torch.tensor(float(pe.numel()), dtype=torch.float64)])
    return (pe, te), red


def edge_k(n_total) -> int:
    return int(float(n_total) * 0.1)  # modules/trainer.py:176: int(numel * 0.1)


def edge_state(red):
    """Radix-select state of both maps: [prefix bits, elements still to take]."""
    k = edge_k(red[4])
    return [[0, k], [0, k]]


def _bits(x):
    return x.contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF


def edge_hist(maps, pass_, state):
    """256-bin histogram of bits [shift, shift+8) of the elements whose higher bits equal the
    selected prefix, for each map (positive floats order like their bit patterns)."""
    shift = 24 - 8 * pass_
    himask = 0 if shift >= 24 else (0xFFFFFFFF << (shift + 8)) & 0xFFFFFFFF
    out = []
    for x, (prefix, _) in zip(maps, state):
        u = _bits(x)
        sel = (u & himask) == (prefix & himask)
        out.append(torch.bincount(((u[sel] >> shift) & 255), minlength=256))
    return torch.cat(out)


def edge_select(state, pass_, hist):
    """Pick the bin holding the k-th largest element from the SUMMED histogram."""
    shift = 24 - 8 * pass_
    for q in range(2):
        h = hist[256 * q:256 * (q + 1)].tolist()
        k, cum, b = state[q][1], 0, 255
        while b > 0:
            if cum + h[b] >= k:
                break
            cum += h[b]
            b -= 1
        state[q][0] |= b << shift
        state[q][1] = k - cum


def _tau(prefix):
    return torch.tensor([prefix], dtype=torch.int64).to(torch.int32).view(torch.float32)[0]


def edge_topk(maps, state, red):
    """Per shard: sum of elements above the k-th largest value tau and the count equal to it."""
    for q, (x, (prefix, _)) in enumerate(zip(maps, state)):
        tau = _tau(prefix)
        red[5 + 2 * q] = x[x > tau].double().sum()
        red[6 + 2 * q] = float((x == tau).sum())


def edge_finish(red, state):
    """|d mean| + |d std| + |d mean(top k)|: the top-k mean is (sum above tau + kleft * tau) / k."""
    n, k = red[4], edge_k(red[4])
    mp, sp = _mean_std(red[0], red[1], n)
    mt, st = _mean_std(red[2], red[3], n)
    tkp = (red[5] + state[0][1] * _tau(state[0][0]).double()) / k
    tkt = (red[7] + state[1][1] * _tau(state[1][0]).double()) / k
    return (mp - mt).abs() + (sp - st).abs() + (tkp - tkt).abs()


def region_sharded(shards, threshold, weight, allreduce):
    """shards: [(pred, target, source)] of THIS rank (one per rank in a process group, or
    several emulated ranks with allreduce summing a list)."""
    return region_finish(allreduce([region_partial(p, t, s, threshold) for p, t, s in shards]), weight)


def edge_sharded(shards, allreduce):
    parts = [edge_partial(p, t) for p, t in shards]
    red = allreduce([r for _, r in parts])
    state = edge_state(red)
    for ps in range(4):
        h = allreduce([edge_hist(m, ps, state) for m, _ in parts])
        edge_select(state, ps, h)
    tk = []
    for m, _ in parts:
        r = red.clone()
        edge_topk(m, state, r)
        tk.append(r[5:9])
    red[5:9] = allreduce(tk)
    return edge_finish(red, state)
