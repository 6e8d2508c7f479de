"""Batched weight packs (ops.prepack -> dcs_pack_plan / dcs_pack_batch): every pack the step's layers
ask for, built in two launches from the plans recorded on the weights, equals the per-pack launches
bit for bit — the packed B, its range record, the pre-split fp16 planes of the rows pass and the
window kernels' hi / lo planes with their exponent — for each Generator and PatchGAN geometry
(networks.py: stem with the 4-channel source, stride-2 downs, windowed residual, sub-pixel ups, the
7x7 head, the PatchGAN layers and its 1-channel tail)."""
import pytest
import torch

from test_gpu_ops import rnd

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _arrays(pk):
    out = [pk]
    if hasattr(pk, "_dcs_rng"):
        out.append(pk._dcs_rng[3])
    if hasattr(pk, "_dcs_bh3"):
        out.append(pk._dcs_bh3[1])
    if hasattr(pk, "_dcs_h3"):
        out.extend(pk._dcs_h3)
    return [a.clone() for a in out]


@pytest.mark.parametrize("mode", ["f16x3", "f16"])
def test_prepack_bit_identical(mode):
    from modules.hip import ops
    from modules.hip.lib import DCS_PAD_REFLECT, DCS_PAD_ZERO
    from modules.hip.ops import ConvGeom
    geoms = {
        "stem": (ConvGeom(3, 64, 7, 1, (3, 3, 3, 3), DCS_PAD_REFLECT), [("f", 4), ("d", 1), ("d", 3)]),
        "down1": (ConvGeom(64, 128, 3, 2, (1, 1, 1, 1), DCS_PAD_ZERO), [("f", None), ("d", None)]),
        "res": (ConvGeom(256, 256, 3, 1, (1, 1, 1, 1), DCS_PAD_REFLECT), [("f", None), ("d", None)]),
        "up1": (ConvGeom(256, 128, 3, 1, (1, 1, 1, 1), DCS_PAD_ZERO, up=2), [("f", None), ("d", None)]),
        "head": (ConvGeom(64, 1, 7, 1, (3, 3, 3, 3), DCS_PAD_REFLECT), [("f", None), ("d", None)]),
        "d0": (ConvGeom(1, 64, 4, 2, (1, 1, 1, 1)), [("f", None), ("d", 1)]),
        "d1": (ConvGeom(64, 128, 4, 2, (1, 1, 1, 1)), [("f", None), ("d", None)]),
        "d4": (ConvGeom(512, 1, 4, 1, (2, 2, 1, 1)), [("f", None), ("d", None)]),
    }
    prev = ops.get_mma()
    ops.set_mma(mode)
    try:
        ws, calls = [], []
        for i, (name, (g, plan)) in enumerate(geoms.items()):
            w = (rnd((g.cout, g.cin, g.k, g.k), 70 + i, name + "w") * 0.05).float().to(DEV)
            ws.append(w)
            for kind, arg in plan:
                calls.append((name, w, (g.pack_fwd if kind == "f" else g.pack_dgrad), arg))
        ref = [(name, _arrays(fn(w, arg))) for name, w, fn, arg in calls]
        olds = [fn(w, arg) for name, w, fn, arg in calls]
        assert any(hasattr(p, "_dcs_h3") for p in olds) and any(hasattr(p, "_dcs_bh3") for p in olds)
        for w in ws:
            w.mul_(1.0)  # new version: the cached packs are stale
        ops.prepack(ws)
        for (name, want), (_, w, fn, arg), old in zip(ref, calls, olds):
            pk = fn(w, arg)  # the pack prepack made, found in the cache
            assert pk is not old, name
            got = _arrays(pk)
            assert len(got) == len(want), name
            for a, b in zip(got, want):
                assert torch.equal(a, b), name
    finally:
        ops.set_mma(prev)


def test_prepack_without_plans_is_noop():
    from modules.hip import ops
    w = torch.ones(4, 4, 3, 3, device=DEV)
    ops.prepack([w])  # nothing recorded: no launch, no error
    assert not hasattr(w, "_dcs_packs")
