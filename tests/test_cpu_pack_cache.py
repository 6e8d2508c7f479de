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



def test_fixed_f16x3_layers_switch(monkeypatch):
    """ops._fixed_mma: a stem / head kernel listed in _FIXED_F16X3 (env DUCOSY_F16X3_LAYERS at import) takes
    f16x3 operands in the f16 mode, any other runs in the step's mode; the default list is empty since
    round 6 (every layer on fp16 in config 5's mode)."""
    import os
    import subprocess
    import sys
    from modules.hip import lib, ops
    prev = ops.get_mma()
    try:
        ops.set_mma("f16")
        monkeypatch.setattr(ops, "_FIXED_F16X3", frozenset({"head"}))
        assert ops._fixed_mma("head") == lib.MMA_F16X3
        assert ops._fixed_mma("stem") == lib.MMA_F16
        ops.set_mma("f16x3")
        assert ops._fixed_mma("stem") == lib.MMA_F16X3
    finally:
        ops.set_mma(prev)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = "from modules.hip import ops; print(','.join(sorted(ops._FIXED_F16X3)))"
    for env, want in (("", ""), ("stem,stem_wgrad", "stem,stem_wgrad")):
        e = dict(os.environ, DUCOSY_F16X3_LAYERS=env)
        if env == "":
            e.pop("DUCOSY_F16X3_LAYERS")
        out = subprocess.run([sys.executable, "-c", code], cwd=os.path.join(root, "ducosy-gan_amd"), env=e,
                             capture_output=True, text=True, timeout=300)
        assert out.returncode == 0, out.stderr
        lines = out.stdout.strip().splitlines()
        assert (lines[-1] if lines else "") == want, out.stdout
