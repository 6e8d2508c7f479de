"""Packed-weight cache (ops._cached_pack) on the host: a pack is reused until its weight changes —
an in-place torch write (version counter), or the fused Adam step that writes the parameters behind
the counter and bumps the epoch of exactly the parameters it stepped (modules/optim.py), so the
Discriminator's packs survive the Generator's optimizer step; a global bump invalidates every pack.
Also the plan record prepack walks (ops._record_pack)."""
import torch


def _counter():
    n = [0]

    def make():
        n[0] += 1
        return torch.zeros(1)
    return n, make


def test_pack_cache_per_parameter_epoch():
    from modules.hip import ops
    a, b = torch.ones(4), torch.ones(4)
    na, ma = _counter()
    nb, mb = _counter()
    pa, pb = ops._cached_pack(a, "k", ma), ops._cached_pack(b, "k", mb)
    assert ops._cached_pack(a, "k", ma) is pa and na[0] == 1
    ops.bump_weights_epoch([a])  # a's optimizer stepped
    assert ops._cached_pack(a, "k", ma) is not pa and na[0] == 2
    assert ops._cached_pack(b, "k", mb) is pb and nb[0] == 1  # b's pack survives
    b.mul_(1.0)  # in-place write: version counter
    ops._cached_pack(b, "k", mb)
    assert nb[0] == 2
    ops.bump_weights_epoch()  # global: every pack
    ops._cached_pack(a, "k", ma)
    ops._cached_pack(b, "k", mb)
    assert na[0] == 3 and nb[0] == 3


def test_record_pack_plan():
    from modules.hip import ops
    from modules.hip.ops import ConvGeom
    w = torch.ones(8, 8, 3, 3)
    g = ConvGeom(8, 8, 3, 2, (1, 1, 1, 1))
    ops._record_pack(w, "pack_fwd", g, None)
    ops._record_pack(w, "pack_fwd", g, None)
    ops._record_pack(w, "pack_dgrad", g, 4)
    assert sorted(k[0] for k in w._dcs_plan) == ["pack_dgrad", "pack_fwd"]

