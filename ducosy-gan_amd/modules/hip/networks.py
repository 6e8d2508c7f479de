"""Fused forward/backward of the Generator and Discriminator on the HIP kernels.

Each network is ONE torch.autograd.Function whose forward walks the layers of
modules/model.py:90-131 with the gfx950 kernels and keeps exactly what its hand-written
backward needs.  Fusions relative to the reference's op-by-op eager graph:
  * ReflectionPad / ZeroPad / nearest Upsample / channel concat are folded into the conv
    gathers (never materialised);
  * InstanceNorm(+ReLU/LeakyReLU) of a layer is either materialised once (in_apply) for the
    MFMA convs that consume it in forward AND weight-gradient passes (a per-element prologue
    inside the gather costs those kernels 20-25 %), or applied in the next conv's prologue
    where that is cheap (the LDS-staged narrow head / PatchGAN kernels);
  * biases of convs followed by InstanceNorm are not added (IN removes any per-channel
    constant, so outputs are unchanged) and their gradient is exactly zero;
  * the CBAM tail (channel MLP, spatial attention, residual add) is 3 kernels forward and
    7 backward (modules/hip/ops.py cbam_*).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import torch

from . import ops
from .lib import ACT_AFFINE, ACT_LRELU, ACT_NONE, ACT_RELU, ACT_TANH, DCS_PAD_REFLECT, DCS_PAD_ZERO
from .ops import ConvGeom, Src

# ---------------------------------------------------------------------------------------
# Generator (modules/model.py:90-115)
# ---------------------------------------------------------------------------------------


def gen_layers(cin: int, nb: int):
    return {
        "stem": ConvGeom(cin, 64, 7, 1, (3, 3, 3, 3), DCS_PAD_REFLECT),
        "down1": ConvGeom(64, 128, 3, 2, (1, 1, 1, 1), DCS_PAD_ZERO),
        "down2": ConvGeom(128, 256, 3, 2, (1, 1, 1, 1), DCS_PAD_ZERO),
        "res": ConvGeom(256, 256, 3, 1, (1, 1, 1, 1), DCS_PAD_REFLECT),
        "up1": ConvGeom(256, 128, 3, 1, (1, 1, 1, 1), DCS_PAD_ZERO, up=2),
        "up2": ConvGeom(128, 64, 3, 1, (1, 1, 1, 1), DCS_PAD_ZERO, up=2),
        "head": ConvGeom(64, 1, 7, 1, (3, 3, 3, 3), DCS_PAD_REFLECT),
    }


def gen_param_names(nb: int, use_cbam: bool) -> Dict[str, str]:
    n = {"stem.w": "model.1.weight", "stem.b": "model.1.bias",
         "down1.w": "model.4.weight", "down1.b": "model.4.bias",
         "down2.w": "model.7.weight", "down2.b": "model.7.bias"}
    for b in range(nb):
        p = f"model.{10 + b}"
        n[f"r{b}.c1.w"] = f"{p}.block.1.weight"
        n[f"r{b}.c1.b"] = f"{p}.block.1.bias"
        n[f"r{b}.c2.w"] = f"{p}.block.5.weight"
        n[f"r{b}.c2.b"] = f"{p}.block.5.bias"
        if use_cbam:
            n[f"r{b}.fc1"] = f"{p}.cbam.channel_attention.fc.0.weight"
            n[f"r{b}.fc2"] = f"{p}.cbam.channel_attention.fc.2.weight"
            n[f"r{b}.sa"] = f"{p}.cbam.spatial_attention.conv.weight"
    u = 10 + nb
    n.update({"up1.w": f"model.{u + 1}.weight", "up1.b": f"model.{u + 1}.bias",
              "up2.w": f"model.{u + 5}.weight", "up2.b": f"model.{u + 5}.bias",
              "head.w": f"model.{u + 9}.weight", "head.b": f"model.{u + 9}.bias"})
    return n


# the InstanceNorm backward's partial sums of each residual block's first IN fused into the data
# gradient that produces its input gradient (window path); False = separate partial-sum pass
_FUSE_IBW = True

# parameter gradients written in place into freshly zeroed .grad buffers; False = always through autograd
_GRAD_SINK = True
# a second contribution to an existing .grad (the model called twice in one step) written to scratch
# and added by one multi-tensor launch at the end of the backward; False = through autograd's adds
_GRAD_ACC = True


class _GradSink:
    """Parameter gradients of one backward pass.  A parameter whose ``.grad`` the fused optimizer has
    just zeroed (modules/optim.py FusedAdam.zero_grad stamps it ``_dcs_fresh`` with the .grad's address
    and version counter) receives its gradient in place while the stamp still matches: the producing
    kernel writes straight into ``.grad`` and autograd gets None, so there is no AccumulateGrad add and
    no zero fill.  Any other parameter (the second batched G_A2B call of a step, a .grad some torch op
    wrote to since the zeroing, plain ``.backward()`` without the fused optimizer) gets its gradient
    added: to scratch and one multi-tensor add, or back through autograd."""

    def __init__(self, params):
        self.params = params or {}
        self.out = {}
        self.acc = []  # (scratch, .grad) pairs: second contributions, added by finish()

    def dest(self, k, view=None) -> Optional[torch.Tensor]:
        p = self.params.get(k)
        g = None if (p is None or not _GRAD_SINK) else p.grad
        if g is None or not g.is_contiguous() or g.dtype != torch.float32:
            return None
        stamp = getattr(p, "_dcs_fresh", None)
        p._dcs_fresh = None
        if stamp is not None and stamp == (g.data_ptr(), g._version):
            return g if view is None else g.view(view)
        if not _GRAD_ACC:
            return None
        s = torch.empty_like(g)  # every producer overwrites its destination
        self.acc.append((s, g))
        return s if view is None else s.view(view)

    def finish(self):
        """Add the second contributions into their .grad buffers (one launch per 64 tensors)."""
        ops.multi_add(self.acc)
        self.acc = []

    def put(self, k, fn, view=None):
        d = self.dest(k, view)
        r = fn(d)
        self.out[k] = None if d is not None else r

    def zero(self, k, like, device=None):
        """A bias an InstanceNorm follows: exact zero gradient (nothing to add to an existing .grad).
        ``like``: a tensor of the bias' shape, or the shape (with ``device``)."""
        p = self.params.get(k)
        if p is not None and p.grad is not None:
            self.out[k] = None
        elif torch.is_tensor(like):
            self.out[k] = torch.zeros_like(like)
        else:
            self.out[k] = torch.zeros(like, device=device, dtype=torch.float32)

    def get(self, k):
        return self.out.get(k)


class _Block:
    __slots__ = ("x", "y1", "s1", "a1", "y2", "s2", "cb")


def _res_block_forward(L, W, b, x, use_cbam, keep):
    """One ResidualBlock[WithCBAM] (modules/model.py:56-87) on NHWC x.  The IN + ReLU between the
    two convs is materialised once (in_apply) for conv2's forward and weight gradient: applying it
    in the window kernels' staging instead measured 1.3 ms per step slower (profiles/r03h)."""
    res = L["res"]
    y1, s1 = res.forward_in_stats(Src.nhwc(x), W["pk"][f"r{b}.c1.w"])
    a1 = ops.in_apply(y1, s1, ACT_RELU)
    y2, s2 = res.forward_in_stats(Src.nhwc(a1), W["pk"][f"r{b}.c2.w"], want_max=use_cbam)
    cb = None
    if use_cbam:
        w1, w2, wsa = W[f"r{b}.fc1"], W[f"r{b}.fc2"], W[f"r{b}.sa"]
        out, cb = ops.cbam_forward(x, y2, s2, w1.reshape(w1.shape[0], -1), w2.reshape(w2.shape[0], -1),
                                   wsa.reshape(2, wsa.shape[-2], wsa.shape[-1]))
    else:
        out = ops.in_apply(y2, s2, ACT_AFFINE)
        ops.scale_add_(out, x)
    blk = None
    if keep:
        blk = _Block()
        blk.x, blk.y1, blk.s1, blk.a1, blk.y2, blk.s2, blk.cb = x, y1, s1, a1, y2, s2, cb
    return out, blk


def _res_block_backward(L, W, b, blk, dout, use_cbam, grads):
    res = L["res"]
    if use_cbam:
        w1, w2, wsa = W[f"r{b}.fc1"], W[f"r{b}.fc2"], W[f"r{b}.sa"]
        k1, k2, k3 = f"r{b}.fc1", f"r{b}.fc2", f"r{b}.sa"
        w1m, w2m, wsam = (w1.reshape(w1.shape[0], -1), w2.reshape(w2.shape[0], -1),
                          wsa.reshape(2, wsa.shape[-2], wsa.shape[-1]))
        o = (grads.dest(k1, w1m.shape), grads.dest(k2, w2m.shape), grads.dest(k3, wsam.shape))
        dy2, dw1, dw2, dwsa = ops.cbam_backward(dout, blk.y2, blk.s2, w1m, w2m, wsam, blk.cb, out_dw=o)
        grads.out[k1] = None if o[0] is not None else dw1.view_as(w1)
        grads.out[k2] = None if o[1] is not None else dw2.view_as(w2)
        grads.out[k3] = None if o[2] is not None else dwsa.view_as(wsa)
    else:
        dy2 = ops.in_act_backward(dout, blk.y2, blk.s2, ACT_AFFINE)
    H, Wd = blk.x.shape[1], blk.x.shape[2]
    grads.put(f"r{b}.c2.w", lambda o: res.wgrad(dy2, Src.nhwc(blk.a1), out=o))
    if _FUSE_IBW:  # IN1's backward partial sums from the data gradient's epilogue (window path)
        da1, parts, nch = res.dgrad(dy2, res.pack_dgrad(W[f"r{b}.c2.w"]), H, Wd, inbwd=(blk.y1, blk.s1, ACT_RELU))
        if parts is not None:
            dy1 = ops.in_act_backward_parts(da1, blk.y1, blk.s1, ACT_RELU, parts, nch)
        else:
            dy1 = ops.in_act_backward(da1, blk.y1, blk.s1, ACT_RELU)
    else:
        da1 = res.dgrad(dy2, res.pack_dgrad(W[f"r{b}.c2.w"]), H, Wd)
        dy1 = ops.in_act_backward(da1, blk.y1, blk.s1, ACT_RELU)
    del da1
    grads.put(f"r{b}.c1.w", lambda o: res.wgrad(dy1, Src.nhwc(blk.x), out=o))
    # residual: dx = dout + dgrad(conv1)
    return res.dgrad(dy1, res.pack_dgrad(W[f"r{b}.c1.w"]), H, Wd, addend=dout)


def _down_forward(g, y, st, wpack):
    """Down-conv over a = relu(IN(y)), materialised by in_apply.  (Staging the IN + ReLU as a
    prologue of the down-conv's forward and weight gradient instead was measured 1.5 ms per step
    slower, profiles/r04an/, and removed.)"""
    a = ops.in_apply(y, st, ACT_RELU)
    out, so = g.forward_in_stats(Src.nhwc(a), wpack)
    return out, so, a


def _down_wgrad(g, dy, y, st, a, o):
    return g.wgrad(dy, Src.nhwc(a), out=o)


def generator_forward(W: Dict[str, torch.Tensor], x: torch.Tensor, x2: Optional[torch.Tensor],
                      nb: int, use_cbam: bool, keep: bool):
    """x: NCHW image (or full concat input); x2: optional NCHW mask channels (concat fused).
    Returns (out [N,1,H,W], saved or None)."""
    cin = x.shape[1] + (x2.shape[1] if x2 is not None else 0)
    L = gen_layers(cin, nb)
    W = dict(W)
    W["pk"] = pk = {}
    for name in ("down1", "down2", "up1", "up2", "head"):
        pk[f"{name}.w"] = L[name].pack_fwd(W[f"{name}.w"])
    # stem input: image (+ mask planes) packed once into NHWC x 4 channels, so the 7x7 gather
    # moves one float4 per tap (the reference's torch.cat of image and masks, fused)
    stem_src = Src.nhwc(ops.pack_nhwc4(x, x2)) if cin <= 4 else Src.nchw(x, x2)
    pk["stem.w"] = L["stem"].pack_fwd(W["stem.w"], cin_pad=stem_src.C)
    for b in range(nb):
        pk[f"r{b}.c1.w"] = L["res"].pack_fwd(W[f"r{b}.c1.w"])
        pk[f"r{b}.c2.w"] = L["res"].pack_fwd(W[f"r{b}.c2.w"])
    N, H, Wd = stem_src.N, stem_src.H, stem_src.W
    # every conv followed by an InstanceNorm returns its statistics (fused into the conv epilogue)
    y0, s0 = L["stem"].forward_in_stats(stem_src, pk["stem.w"])
    y1, s1, a0 = _down_forward(L["down1"], y0, s0, pk["down1.w"])
    y2, s2, a1 = _down_forward(L["down2"], y1, s1, pk["down2.w"])
    h = ops.in_apply(y2, s2, ACT_RELU)
    blocks = []
    for b in range(nb):
        h, blk = _res_block_forward(L, W, b, h, use_cbam, keep)
        blocks.append(blk)
    yu1, su1 = L["up1"].forward_in_stats(Src.nhwc(h), pk["up1.w"])
    au1 = ops.in_apply(yu1, su1, ACT_RELU)
    yu2, su2 = L["up2"].forward_in_stats(Src.nhwc(au1), pk["up2.w"], want_max=True)
    out = L["head"].forward(Src.nhwc(yu2), pk["head.w"], bias=W["head.b"],
                            pro=(su2.scale, su2.shift, ACT_RELU), epi_act=ACT_TANH, pro_max=su2.xmax)
    out = out.view(N, 1, H, Wd)
    saved = None
    if keep:
        saved = dict(L=L, W=W, xs=stem_src, y0=y0, s0=s0, a0=a0, y1=y1, s1=s1, a1=a1, y2=y2, s2=s2, blocks=blocks,
                     h=h, yu1=yu1, su1=su1, au1=au1, yu2=yu2, su2=su2, nb=nb, use_cbam=use_cbam)
    else:
        del a0, a1, au1
    return out, saved


def _dgrad_in_act(g, dy, w, H, Wd, y, st):
    """dL/dy of a layer a = relu(IN(y)) whose activation feeds conv g: g's data gradient, then the IN +
    ReLU backward; the backward's partial sums come from the data gradient's epilogue where the window
    phase kernels run it (ConvGeom.dgrad(..., inbwd=...))."""
    if _FUSE_IBW:
        da, parts, nch = g.dgrad(dy, g.pack_dgrad(w), H, Wd, inbwd=(y, st, ACT_RELU))
        if parts is not None:
            return ops.in_act_backward_parts(da, y, st, ACT_RELU, parts, nch)
    else:
        da = g.dgrad(dy, g.pack_dgrad(w), H, Wd)
    return ops.in_act_backward(da, y, st, ACT_RELU)


def generator_backward(S, dout: torch.Tensor, need_dx: bool, dx_channels: int, dx_from: int = 0,
                       params: Optional[Dict[str, torch.Tensor]] = None, slice_only: bool = False):
    """Returns (dx NHWC [N,H,W,dx_channels] or None, _GradSink keyed like gen_param_names: .get(k)
    is the gradient to hand to autograd, None where it went into the parameter's .grad in place).
    dx is computed for samples dx_from.. only (zero before; with slice_only, dx holds those samples
    only: [N - dx_from, H, W, dx_channels], no zero fill)."""
    L, W = S["L"], S["W"]
    nb, use_cbam = S["nb"], S["use_cbam"]
    grads = _GradSink(params)
    N, _, H, Wd = dout.shape
    dout = dout.contiguous()
    # head: tanh backward, bias, wgrad, dgrad
    dpre = ops.act_backward(dout, S["out"], ACT_TANH).view(N, H, Wd, 1)
    grads.put("head.b", lambda o: ops.channel_sum(dpre, out=o))
    su2, su1 = S["su2"], S["su1"]
    grads.put("head.w", lambda o: L["head"].wgrad(dpre, Src.nhwc(S["yu2"]), pro=(su2.scale, su2.shift, ACT_RELU),
                                                   out=o, pro_max=su2.xmax))
    wk = L["head"].pack_dgrad(W["head.w"])
    dy = ops.head_dgrad_in(dpre, wk, S["yu2"], su2, ACT_RELU)
    if dy is None:
        da = L["head"].dgrad(dpre, wk, H, Wd)
        dy = ops.in_act_backward(da, S["yu2"], su2, ACT_RELU)
    del dpre
    # up2
    grads.put("up2.w", lambda o: L["up2"].wgrad(dy, Src.nhwc(S["au1"]), out=o))
    # up1's input gradient: up2's data gradient with the IN + ReLU backward's partial sums fused where the
    # window phase kernels run it
    dy = _dgrad_in_act(L["up2"], dy, W["up2.w"], H // 2, Wd // 2, S["yu1"], su1)
    grads.put("up1.w", lambda o: L["up1"].wgrad(dy, Src.nhwc(S["h"]), out=o))
    dh = L["up1"].dgrad(dy, L["up1"].pack_dgrad(W["up1.w"]), H // 4, Wd // 4)
    del dy
    # residual blocks
    for b in reversed(range(nb)):
        dh = _res_block_backward(L, W, b, S["blocks"][b], dh, use_cbam, grads)
        S["blocks"][b] = None
    # x0 = relu(IN(y2))
    s2, s1, s0 = S["s2"], S["s1"], S["s0"]
    dy = ops.in_act_backward(dh, S["y2"], s2, ACT_RELU)
    grads.put("down2.w", lambda o: _down_wgrad(L["down2"], dy, S["y1"], s1, S["a1"], o))
    dy = _dgrad_in_act(L["down2"], dy, W["down2.w"], H // 2, Wd // 2, S["y1"], s1)
    grads.put("down1.w", lambda o: _down_wgrad(L["down1"], dy, S["y0"], s0, S["a0"], o))
    dy = _dgrad_in_act(L["down1"], dy, W["down1.w"], H, Wd, S["y0"], s0)
    grads.put("stem.w", lambda o: L["stem"].wgrad(dy, S["xs"], out=o))
    dx = None
    if need_dx:
        stem = L["stem"]
        wd = stem.pack_dgrad(W["stem.w"], dx_channels)
        if dx_from > 0 and slice_only:
            dx = stem.dgrad(dy[dx_from:], wd, H, Wd, ci_count=dx_channels)
        elif dx_from > 0:
            dx = torch.zeros(N, H, Wd, dx_channels, device=dy.device, dtype=torch.float32)
            if dx_from < N:
                dx[dx_from:] = stem.dgrad(dy[dx_from:], wd, H, Wd, ci_count=dx_channels)
        else:
            dx = stem.dgrad(dy, wd, H, Wd, ci_count=dx_channels)
    # biases feeding an InstanceNorm: exact zero gradient
    for key in ("stem.b", "down1.b", "down2.b", "up1.b", "up2.b"):
        grads.zero(key, W[key])
    for b in range(nb):
        grads.zero(f"r{b}.c1.b", W[f"r{b}.c1.b"])
        grads.zero(f"r{b}.c2.b", W[f"r{b}.c2.b"])
    grads.finish()
    return dx, grads


class GeneratorFunction(torch.autograd.Function):
    """out = Generator(x [, x2]) with a fused hand-written backward."""

    @staticmethod
    def forward(ctx, x, x2, cfg, *params):
        keys, nb, use_cbam = cfg[:3]
        ctx.dx_from = cfg[3] if len(cfg) > 3 else 0
        W = dict(zip(keys, params))
        keep = any(ctx.needs_input_grad)
        out, saved = generator_forward(W, x, x2, nb, use_cbam, keep)
        ctx.saved = saved
        if keep:
            ctx.save_for_backward(out)  # tanh backward needs the output (no ctx attribute cycle)
            # the parameters themselves: freshly zeroed .grad buffers take their gradients in place
            ctx.params = {k: p for i, (k, p) in enumerate(zip(keys, params)) if ctx.needs_input_grad[3 + i]}
        ctx.keys = keys
        ctx.x_channels = x.shape[1]
        return out

    @staticmethod
    def backward(ctx, dout):
        S = ctx.saved
        S["out"] = ctx.saved_tensors[0]
        need_dx = ctx.needs_input_grad[0]
        dx_nhwc, grads = generator_backward(S, dout, need_dx, ctx.x_channels, ctx.dx_from, ctx.params)
        ctx.saved = None
        ctx.params = None
        dx = None
        if need_dx:
            dx = dx_nhwc.permute(0, 3, 1, 2)
            if ctx.x_channels > 1:
                dx = dx.contiguous()
        dparams = [grads.get(k) if ctx.needs_input_grad[3 + i] else None for i, k in enumerate(ctx.keys)]
        return (dx, None, None, *dparams)


# ---------------------------------------------------------------------------------------
# Discriminator (modules/model.py:118-131)
# ---------------------------------------------------------------------------------------

def disc_layers(cin: int):
    return [ConvGeom(cin, 64, 4, 2, (1, 1, 1, 1)), ConvGeom(64, 128, 4, 2, (1, 1, 1, 1)),
            ConvGeom(128, 256, 4, 2, (1, 1, 1, 1)), ConvGeom(256, 512, 4, 2, (1, 1, 1, 1)),
            ConvGeom(512, 1, 4, 1, (2, 2, 1, 1))]  # ZeroPad2d((1,0,1,0)) + padding=1


DISC_KEYS = ["model.0.weight", "model.0.bias", "model.2.weight", "model.2.bias", "model.5.weight",
             "model.5.bias", "model.8.weight", "model.8.bias", "model.12.weight", "model.12.bias"]


_UNIT = {}


def _unit_affine(N: int, dev) -> tuple:
    """(ones, zeros) [N, 64]: the identity prologue of PatchGAN layer 1 (read-only, cached)."""
    key = (N, str(dev))
    if key not in _UNIT:
        _UNIT[key] = (torch.ones(N, 64, device=dev, dtype=torch.float32),
                      torch.zeros(N, 64, device=dev, dtype=torch.float32))
    return _UNIT[key]


def discriminator_forward(params: List[torch.Tensor], x: torch.Tensor, keep: bool):
    L = disc_layers(x.shape[1])
    ws = params[0::2]
    bs = params[1::2]
    # layer-0 input packed NHWC x 4 (zero channels) for the vectorised gather
    xs = Src.nhwc(ops.pack_nhwc4(x)) if x.shape[1] <= 4 else Src.nchw(x)
    pk = [L[0].pack_fwd(ws[0], cin_pad=xs.C)] + [g.pack_fwd(w) for g, w in zip(L[1:], ws[1:])]
    N = x.shape[0]
    dev = x.device
    # layer 0: conv + bias; its LeakyReLU is the next conv's prologue (scale 1, shift 0)
    y0 = L[0].forward(xs, pk[0], bias=bs[0])
    ones, zeros = _unit_affine(N, dev)
    ys, sts = [y0], [ops.INStats(ones, zeros)]
    h = y0
    for i in (1, 2, 3):
        st = sts[-1]
        h, st = L[i].forward_in_stats(Src.nhwc(h), pk[i], pro=(st.scale, st.shift, ACT_LRELU))
        ys.append(h)
        sts.append(st)
    st = sts[-1]
    out = L[4].forward(Src.nhwc(h), pk[4], bias=bs[4], pro=(st.scale, st.shift, ACT_LRELU))
    H4, W4 = out.shape[1], out.shape[2]
    out = out.view(N, 1, H4, W4)
    saved = dict(L=L, ws=ws, xs=xs, ys=ys, sts=sts) if keep else None
    return out, saved


def discriminator_backward(S, dout, need_dx, need_w, params=None):
    """Returns (dx or None, _GradSink keyed 0..9 in DISC_KEYS order)."""
    L, ws, ys, sts = S["L"], S["ws"], S["ys"], S["sts"]
    N, _, H4, W4 = dout.shape
    d = dout.contiguous().view(N, H4, W4, 1)
    grads = _GradSink(params)
    if need_w:
        grads.put(9, lambda o: ops.channel_sum(d, out=o))
        st = sts[3]
        grads.put(8, lambda o: L[4].wgrad(d, Src.nhwc(ys[3]), pro=(st.scale, st.shift, ACT_LRELU), out=o))
    da = L[4].dgrad(d, L[4].pack_dgrad(ws[4]), ys[3].shape[1], ys[3].shape[2])
    for i in (3, 2, 1):
        dy = ops.in_act_backward(da, ys[i], sts[i], ACT_LRELU)
        if need_w:
            st = sts[i - 1]
            grads.put(2 * i, lambda o: L[i].wgrad(dy, Src.nhwc(ys[i - 1]), pro=(st.scale, st.shift, ACT_LRELU), out=o))
            grads.zero(2 * i + 1, (L[i].cout,), d.device)
        da = L[i].dgrad(dy, L[i].pack_dgrad(ws[i]), ys[i - 1].shape[1], ys[i - 1].shape[2])
    # layer 0: y0 includes the bias; a0 = lrelu(y0)
    dy0 = ops.act_backward(da, ys[0], ACT_LRELU)
    if need_w:
        grads.put(1, lambda o: ops.channel_sum(dy0, out=o))
        grads.put(0, lambda o: L[0].wgrad(dy0, S["xs"], out=o))
    dx = None
    if need_dx:
        xs = S["xs"]
        dx = L[0].dgrad(dy0, L[0].pack_dgrad(ws[0]), xs.H, xs.W)
    grads.finish()
    return dx, grads


class DiscriminatorFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, *params):
        keep = any(ctx.needs_input_grad)
        out, saved = discriminator_forward(list(params), x, keep)
        ctx.saved = saved
        ctx.params = {i: p for i, p in enumerate(params) if ctx.needs_input_grad[1 + i]} if keep else None
        return out

    @staticmethod
    def backward(ctx, dout):
        need_dx = ctx.needs_input_grad[0]
        need_w = any(ctx.needs_input_grad[1:])
        dx, grads = discriminator_backward(ctx.saved, dout, need_dx, need_w, ctx.params)
        ctx.saved = None
        ctx.params = None
        if dx is not None:
            dx = dx.permute(0, 3, 1, 2)
            if dx.shape[1] > 1:
                dx = dx.contiguous()
        return (dx, *[grads.get(i) if ctx.needs_input_grad[1 + i] else None for i in range(10)])


class ResBlockFunction(torch.autograd.Function):
    """Standalone ResidualBlock[WithCBAM] (modules/model.py:56-87) on an NCHW tensor."""

    @staticmethod
    def forward(ctx, x, use_cbam, keys, *params):
        W = dict(zip(keys, params))
        L = {"res": ConvGeom(x.shape[1], x.shape[1], 3, 1, (1, 1, 1, 1), DCS_PAD_REFLECT)}
        W["pk"] = {"r0.c1.w": L["res"].pack_fwd(W["r0.c1.w"]), "r0.c2.w": L["res"].pack_fwd(W["r0.c2.w"])}
        xh = x.permute(0, 2, 3, 1).contiguous()
        keep = any(ctx.needs_input_grad)
        out, blk = _res_block_forward(L, W, 0, xh, use_cbam, keep)
        ctx.state = (L, W, blk, use_cbam, keys) if keep else None
        return out.permute(0, 3, 1, 2).contiguous()

    @staticmethod
    def backward(ctx, dout):
        L, W, blk, use_cbam, keys = ctx.state
        grads = _GradSink(None)
        dx = _res_block_backward(L, W, 0, blk, dout.permute(0, 2, 3, 1).contiguous(), use_cbam, grads)
        grads.zero("r0.c1.b", W["r0.c1.b"])
        grads.zero("r0.c2.b", W["r0.c2.b"])
        ctx.state = None
        return (dx.permute(0, 3, 1, 2).contiguous(), None, None,
                *[grads.get(k) if ctx.needs_input_grad[3 + i] else None for i, k in enumerate(keys)])
