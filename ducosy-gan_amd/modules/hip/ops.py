"""Tensor-level wrappers over the C-ABI (device pointers, shapes, workspaces, streams).

PyTorch is plumbing here: it owns device memory (caching allocator) and the stream; every
arithmetic op on the hot path is one of the hand-written gfx950 kernels behind lib.py.
Activations are NHWC fp32 contiguous tensors.
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass
from typing import Optional, Tuple

import torch

from . import lib
from .lib import ACT_AFFINE, ACT_LRELU, ACT_NONE, ACT_RELU, ACT_TANH, DCS_PAD_REFLECT, DCS_PAD_ZERO

IN_EPS = 1e-5

# MFMA operand mode of the MFMA convolution passes (include/ducosy_hip.h DCS_MMA_*): "f32" is
# exact fp32 (the reference's precision); "f16x3" / "bf16x6" split each fp32 operand into fp16 / bf16
# parts (fp32-class); "f16" rounds the power-of-two scaled operands to fp16 and "bf16" to bf16
# (BASELINE config 5's half-precision path); "bf16x3" splits each operand into hi + lo bf16.
_MMA_NAMES = {"f32": lib.MMA_F32, "bf16": lib.MMA_BF16, "bf16x3": lib.MMA_BF16X3, "bf16x6": lib.MMA_BF16X6,
              "f16x3": lib.MMA_F16X3, "f16": lib.MMA_F16}
# default f16x3: fp32-class (max error vs float64 <= the exact-f32 MFMA path's on every layer,
# tests/test_gpu_mma.py::test_bf16x6_error_matches_exact_f32, also for bf16x6) at half of bf16x6's MFMAs
_MMA = _MMA_NAMES[os.environ.get("DUCOSY_MMA", "f16x3")]
# Path selectors below are module constants, not environment switches: the tests flip them (e.g.
# ops._WIN = False) to hold a fused path to the one it replaced.
# the Generator head's forward by tap projection on the MFMA pipe in the fp16 modes
# (csrc/conv_head.hip); False = the exact-f32 VALU kernel
_HEAD_PROJ = True
_BPRE = True  # pre-split fp16 weight planes for the f16x3 / f16 rows pass
_STEM = True  # the Generator stem on its MFMA kernel (csrc/conv_stem.hip)
_PREPACK = True  # the step's weight packs in two batched launches
_SUBWIN = True  # up-conv forwards on the sub-pixel window kernel
_SUBWIN_D = True  # (diagnostic: their data gradients too)
_S2WIN = True  # the down-convs on the same window phase kernels


# residual convs in the slice-major K order (DCS_KORDER_SLICE); False = tap-major
# IN statistics fused into the conv epilogue (ConvGeom.forward_in_stats); False = separate pass
_FUSE_STATS = True
_KSLICE = True
# reflection fold of the stride-1 pad-1 data gradient in the conv epilogue (dcs_conv_dgrad_reflect);
# False = padded-grid rows pass + dcs_reflect_fold
_FUSE_FOLD = True
# f16x3 residual convs on the window kernel (csrc/conv_win.hip); False = the rows pass
_WIN = True
# window phase-kernel layers kept on f16x3 operands in the fp16 mode (ConvGeom._phase_tag).  Empty since
# round 6: every up-conv and PatchGAN layer on fp16 operands holds the config-5 bars (the steps_64 fixture
# pair at 0.60 of its bar, the 512 x 512 pair within 1.4e-4 / 3.7e-3 of f16x3; scripts/diag/f16_layers.py,
# profiles/r06/ab/r06ab_*), f16 step 138.7 -> 133.5 ms same box
_PHASE_F16X3 = frozenset()
# the Generator's stem and head kernels kept on f16x3 operands in the fp16 mode ("stem": forward, "stem_wgrad",
# "head": forward, data and weight gradient); a layer left out runs in the step's mode (env DUCOSY_F16X3_LAYERS:
# a comma-separated list in place of the default).  Empty since round 6: with every layer on fp16 the steps_64
# fixture pair holds 0.74 of its bar (0.67 with the three kept; scripts/diag/f16_layers.py --fixed), f16 step
# 131.3 -> 130.3 ms same box (profiles/r06/ab/r06ai_*)
_FIXED_F16X3 = frozenset(x for x in os.environ.get("DUCOSY_F16X3_LAYERS", "").split(",") if x)


def _fixed_mma(layer: str) -> int:
    return lib.MMA_F16X3 if layer in _FIXED_F16X3 else _MMA


def _h3() -> bool:
    """f16x3 or f16: the power-of-two scaled fp16 operand modes (range records, window kernels)."""
    return _MMA in (lib.MMA_F16X3, lib.MMA_F16)


def _fallback() -> int:
    """Mode of a pass the fp16 kernels do not cover (no range record: concat or strided sources):
    bf16x6 under f16x3 (fp32-class), plain bf16 under f16 (half precision)."""
    return lib.MMA_BF16 if _MMA == lib.MMA_F16 else lib.MMA_BF16X6


def set_mma(mode: str) -> None:
    global _MMA
    if mode not in _MMA_NAMES:
        raise ValueError(f"mma mode must be one of {sorted(_MMA_NAMES)}")
    _MMA = _MMA_NAMES[mode]


def get_mma() -> str:
    return {v: k for k, v in _MMA_NAMES.items()}[_MMA]


def _p(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _ptr(t: Optional[torch.Tensor]):
    return t.data_ptr() if t is not None else None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _check_dev(*ts):
    for t in ts:
        if t is not None:
            if not t.is_cuda:
                raise RuntimeError("ducosy HIP ops require device tensors (no CPU fallback)")
            if t.dtype not in (torch.float32, torch.int32, torch.uint8):
                raise RuntimeError(f"unsupported dtype {t.dtype}")


# ---------------------------------------------------------------------------------------
# workspace
# ---------------------------------------------------------------------------------------
_WS = {}
_WS_POISON = os.environ.get("DUCOSY_WS_POISON", "0") == "1"


def workspace(nbytes: int, device) -> torch.Tensor:
    """Scratch buffer reused across calls: one per (device, stream), so stream-ordered reuse is
    safe and models stepping concurrently on different streams never share scratch."""
    nbytes = max(int(nbytes), 256)
    dev = torch.device(device)
    key = (dev.index, torch.cuda.current_stream(dev).cuda_stream)
    buf = _WS.get(key)
    if buf is None or buf.numel() < nbytes:
        size = max(nbytes, int(buf.numel() * 1.5) if buf is not None else 0)
        buf = torch.empty(size, dtype=torch.uint8, device=device)
        _WS[key] = buf
    if _WS_POISON:  # debug: every request sees NaN bytes (finds reads of unwritten scratch)
        buf.fill_(0xFF)
    return buf


def _round_up(x, m):
    return (x + m - 1) // m * m


# ---------------------------------------------------------------------------------------
# f16x3 operand range records (include/ducosy_hip.h DCS_MMA_F16X3, dcs_range_parts)
# ---------------------------------------------------------------------------------------
# Range-record arena per (device, stream): producers' records are slots of one buffer, zeroed in one
# launch when the arena is reset (range_arena_reset, once per training step) instead of one memset
# per record (include/ducosy_hip.h dcs_range_arena_register).  A record remembers the arena
# generation it was handed out in; after a reset it is stale and range_rec recomputes it.
_ARENA = {}
_ARENA_SLOTS = int(os.environ.get("DUCOSY_RANGE_ARENA", "256"))


def _arena(dev):
    key = (dev.index, torch.cuda.current_stream(dev).cuda_stream)
    a = _ARENA.get(key)
    if a is None and _ARENA_SLOTS > 0:
        buf = torch.zeros(_ARENA_SLOTS * lib.RANGE_PARTS, device=dev, dtype=torch.float32)
        lib.call("dcs_range_arena_register", _p(buf), buf.numel() * 4)
        a = _ARENA[key] = [buf, 0, 0, key]  # buffer, next slot, generation, key
    return a


def range_arena_reset(device) -> None:
    """Zero the used records of this stream's arena (one launch) and start a new generation:
    every record handed out before is stale from here on."""
    a = _arena(torch.device(device))
    if a is None:
        return
    if a[1]:
        a[0][:a[1] * lib.RANGE_PARTS].zero_()
    a[1] = 0
    a[2] += 1


def _rng_valid(cached) -> bool:
    if len(cached) < 6 or cached[4] is None:
        return True
    a = _ARENA.get(cached[5])
    return a is not None and a[2] == cached[4]


def range_rec(t: torch.Tensor, pro: Optional[Tuple[torch.Tensor, torch.Tensor, int]] = None) -> torch.Tensor:
    """DCS_RANGE_PARTS partial maxima of |t| (or of |act(t * scale + shift)| with a per-(image,
    channel) prologue) for an NHWC tensor: the f16x3 kernels reduce them to the operand's power-of-two
    scale.  Cached on the tensor object per (version, prologue), so the forward, data-gradient and
    weight-gradient passes over one activation or gradient compute it once."""
    if pro is not None:  # a record from the IN statistics (attach_act_range): no pass over t
        ar = getattr(pro[0], "_dcs_act_rng", None)
        if ar is not None and ar[0] == pro[2] and ar[1] is pro[1]:
            return ar[2]
    cached = getattr(t, "_dcs_rng", None)
    if cached is not None and cached[0] == t._version and cached[1] is (pro[0] if pro else None) \
            and cached[2] == (pro[2] if pro else ACT_NONE) and _rng_valid(cached):
        return cached[3]
    parts = torch.empty(lib.RANGE_PARTS, device=t.device, dtype=torch.float32)
    N, C = t.shape[0], t.shape[-1]
    lib.call("dcs_range_parts", _p(t), N, t.numel() // N, C, _p(pro[0]) if pro else None,
             _p(pro[1]) if pro else None, pro[2] if pro else ACT_NONE, _p(parts), _stream())
    t._dcs_rng = (t._version, pro[0] if pro else None, pro[2] if pro else ACT_NONE, parts)
    return parts


def attach_act_range(st: "INStats", act: int) -> None:
    """The range record of a = act(y * scale + shift) from the IN statistics (per (image, channel) max of
    y, scale > 0): max |a| = max(0, xmax * scale + shift) for ReLU, attached to st.scale for range_rec,
    so a consumer staging a as a prologue reads no extra pass over y."""
    assert act == ACT_RELU and st.xmax is not None
    rec = torch.zeros(lib.RANGE_PARTS, device=st.scale.device, dtype=torch.float32)
    rec[:1] = torch.clamp(torch.addcmul(st.shift, st.xmax, st.scale), min=0).amax().reshape(1)
    st.scale._dcs_act_rng = (act, st.shift, rec)


def _out_rng(out: torch.Tensor):
    """Range record for a producer kernel to fill while it writes ``out`` (f16x3 mode only): the
    kernel zeroes it and folds max |value| in; attached to ``out`` like range_rec's cache."""
    if not _h3():
        return None
    a = _arena(out.device)
    if a is not None and a[1] < _ARENA_SLOTS:  # a pre-zeroed arena slot: the producer skips its memset
        rng = a[0][a[1] * lib.RANGE_PARTS:(a[1] + 1) * lib.RANGE_PARTS]
        a[1] += 1
        out._dcs_rng = (out._version, None, ACT_NONE, rng, a[2], a[3])
    else:
        rng = torch.empty(lib.RANGE_PARTS, device=out.device, dtype=torch.float32)
        out._dcs_rng = (out._version, None, ACT_NONE, rng)
    return _p(rng)


def _drop_rng(t: torch.Tensor) -> None:
    """Forget a range record after an in-place write the autograd version counter cannot see."""
    if hasattr(t, "_dcs_rng"):
        del t._dcs_rng


def _set_mma(d: lib.ConvDesc, a: Optional[torch.Tensor], a_pro, b_rng: Optional[torch.Tensor],
             wpack: Optional[torch.Tensor] = None) -> None:
    """Operand mode of one MFMA pass.  f16x3 needs the range records of both operands: ``a`` (the
    gathered tensor, contiguous, with its prologue) and ``b_rng`` (the packed weights' record, or the
    wgrad source's); a pass without them (concat or strided sources) runs bf16x6.  ``wpack``: the
    rows pass's packed weights, whose pre-split planes (if any) it then stages directly."""
    d.mma = _MMA
    d.b_h3 = None
    if not _h3():
        return
    if a is None or b_rng is None or not a.is_contiguous() or (a.numel() // a.shape[0]) % 4 or a.data_ptr() % 16:
        d.mma = _fallback()
        return
    ra = range_rec(a, a_pro)
    d.rng_a, d.rng_a_n = ra.data_ptr(), ra.numel()
    d.rng_b, d.rng_b_n = b_rng.data_ptr(), b_rng.numel()
    bh = getattr(wpack, "_dcs_bh3", None) if wpack is not None else None
    if bh is not None and bh[0] == wpack._version:
        d.b_h3 = bh[1].data_ptr()


# ---------------------------------------------------------------------------------------
# kernel probe: HIP events around the north-star kernel's launches (bench.py roofline)
# ---------------------------------------------------------------------------------------
class KernelProbe:
    """Records (start, end, algorithmic FLOPs) for every launch of the 256-channel 3x3
    residual-block convolution (conv_rows_kernel<128,128,true,1>: forward and data-gradient)
    on the stream it is launched on, while ``active``."""

    def __init__(self):
        self.active = False
        self.records = []

    def reset(self):
        self.records = []

    def begin(self):
        if not self.active:
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record(torch.cuda.current_stream())
        return e

    def end(self, e0, flops):
        if e0 is None:
            return
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record(torch.cuda.current_stream())
        self.records.append((e0, e1, flops))

    def summary(self):
        """(launches, mean ms per launch, mean algorithmic FLOP per launch)."""
        if not self.records:
            return 0, 0.0, 0.0
        torch.cuda.synchronize()
        ms = [a.elapsed_time(b) for a, b, _ in self.records]
        fl = [f for _, _, f in self.records]
        return len(ms), sum(ms) / len(ms), sum(fl) / len(fl)


PROBE = KernelProbe()


def _is_res_geom(g) -> bool:
    return g.cin == 256 and g.cout == 256 and g.k == 3 and g.stride == 1 and g.up == 1


# ---------------------------------------------------------------------------------------
# convolution geometry
# ---------------------------------------------------------------------------------------
@dataclass
class Src:
    """A gathered operand: logical [N, H, W, C] with element strides; optional second
    tensor supplying channels >= csplit (channel concat fused into the gather)."""
    t: torch.Tensor
    N: int
    H: int
    W: int
    C: int
    strides: Tuple[int, int, int, int]  # (n, c, h, w)
    t2: Optional[torch.Tensor] = None
    strides2: Tuple[int, int, int, int] = (0, 0, 0, 0)
    csplit: Optional[int] = None

    @staticmethod
    def nhwc(t: torch.Tensor) -> "Src":
        N, H, W, C = t.shape
        return Src(t, N, H, W, C, (H * W * C, 1, W * C, C))

    @staticmethod
    def nchw(t: torch.Tensor, t2: Optional[torch.Tensor] = None) -> "Src":
        """NCHW tensor (any strides), optionally concatenated with t2 along channels."""
        N, C, H, W = t.shape
        sn, sc, sh, sw = t.stride()
        if t2 is None:
            return Src(t, N, H, W, C, (sn, sc, sh, sw))
        N2, C2, H2, W2 = t2.shape
        assert (N2, H2, W2) == (N, H, W)
        return Src(t, N, H, W, C + C2, (sn, sc, sh, sw), t2, tuple(t2.stride()), C)


BN_MAX = 128

# Packed-weight cache: a pack is reused while its weight tensor is unchanged -- same autograd version
# and storage (in-place torch ops, load_state_dict, broadcasts bump the version; a .data reassignment
# changes the storage) and same weights epoch (the fused Adam
# kernel writes parameters behind the version counter and bumps the epoch of the parameters it
# stepped, modules/optim.py; a broadcast through a flat buffer bumps the global one).  Within a step
# the second batched G_A2B call and the G-step / D-step Discriminator calls reuse the packs, and the
# Discriminator packs outlive the Generator's optimizer step.
_EPOCH = [0]


def bump_weights_epoch(params=None) -> None:
    """Invalidate the packs of ``params`` (every pack when None)."""
    if params is None:
        _EPOCH[0] += 1
        return
    for p in params:
        p._dcs_epoch = getattr(p, "_dcs_epoch", 0) + 1


def _cached_pack(w: torch.Tensor, key, make):
    stamp = (w.data_ptr(), w._version, _EPOCH[0], getattr(w, "_dcs_epoch", 0), _MMA, _WIN, _KSLICE)
    c = getattr(w, "_dcs_packs", None)
    if c is None or c[0] != stamp:
        c = (stamp, {})
        w._dcs_packs = c
    pk = c[1].get(key)
    if pk is None:
        pk = make()
        c[1][key] = pk
    return pk


class _PackBatch:
    """The weight packs of one prepack call, launched as two batched kernels (dcs_pack_batch)."""
    _pinned = []  # staging buffers of the last few batches (their async copies may still be in flight)

    def __init__(self):
        self.jobs = []
        self.keep = []

    def add(self, w, **kw):
        j = lib.PackJob()
        j.w = w.data_ptr()
        for k, v in kw.items():
            if torch.is_tensor(v):
                self.keep.append(v)  # alive until the launches are queued (the h3 scratch has no other owner)
            setattr(j, k, v.data_ptr() if torch.is_tensor(v) else (0 if v is None else v))
        self.jobs.append(j)
        self.keep.append(w)

    def flush(self, device):
        if not self.jobs:
            return
        n = len(self.jobs)
        arr = (lib.PackJob * n)(*self.jobs)
        g1, g2 = ctypes.c_int(0), ctypes.c_int(0)
        lib.call("dcs_pack_plan", ctypes.addressof(arr), n, ctypes.byref(g1), ctypes.byref(g2))
        nbytes = ctypes.sizeof(arr)
        host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        ctypes.memmove(host.data_ptr(), ctypes.addressof(arr), nbytes)
        dev = host.to(device, non_blocking=True)
        _PackBatch._pinned = (_PackBatch._pinned + [host])[-8:]
        lib.call("dcs_pack_batch", _p(dev), n, g1.value, g2.value, _stream())


_BATCH: Optional[_PackBatch] = None


def _record_pack(w: torch.Tensor, method: str, geom, arg) -> None:
    plan = getattr(w, "_dcs_plan", None)
    if plan is None:
        plan = {}
        w._dcs_plan = plan
    plan.setdefault((method, geom._key(), arg), geom)


def prepack(params) -> None:
    """Every pack a training step will ask for (the pack_fwd / pack_dgrad calls recorded on each
    weight by earlier steps), for the weights' current values, in two batched launches instead of
    one or two small launches per pack at first use.  The packs land in the same cache, so the
    step's own calls find them; their values equal the per-pack calls'."""
    global _BATCH
    if _BATCH is not None or not _PREPACK:
        return
    b = _PackBatch()
    dev = None
    _BATCH = b
    try:
        for w in params:
            plan = getattr(w, "_dcs_plan", None)
            if not plan:
                continue
            dev = w.device
            for (method, _, arg), geom in list(plan.items()):
                getattr(geom, method)(w, arg)
    finally:
        _BATCH = None
    if dev is not None:
        b.flush(dev)


def _wrng(wpack: torch.Tensor) -> Optional[torch.Tensor]:
    """Range record a packed weight tensor carries (dcs_pack_weights_r), None if packed without."""
    r = getattr(wpack, "_dcs_rng", None)
    return r[3] if r is not None and r[0] == wpack._version else None


def _bn_for(co: int) -> int:
    return 128 if co > 64 else 64


@dataclass
class ConvGeom:
    """One nn.Conv2d of the reference with its padding module folded in."""
    cin: int
    cout: int
    k: int
    stride: int = 1
    pads: Tuple[int, int, int, int] = (0, 0, 0, 0)  # top, left, bottom, right
    pad_mode: int = DCS_PAD_ZERO
    up: int = 1  # nearest upsampling of the input before the conv

    @property
    def kslice(self) -> bool:
        """The residual convs run the slice-major K order (include/ducosy_hip.h
        DCS_KORDER_SLICE: 3.7x fewer L2 misses on the gathered rows, 4 % faster in bf16x6) in the
        bf16 operand modes; their packed weights follow it.  The exact-f32 kernel keeps the
        tap-major order (its gather decodes the tap once per 8 k-tiles there)."""
        return _is_res_geom(self) and _KSLICE and _MMA != lib.MMA_F32

    def out_hw(self, H, W):
        Hv, Wv = H * self.up, W * self.up
        t, l, b, r = self.pads
        return (Hv + t + b - self.k) // self.stride + 1, (Wv + l + r - self.k) // self.stride + 1

    @property
    def narrow(self):
        return self.cout <= 4

    @property
    def subpixel(self) -> bool:
        """Nearest-x2 upsample + 3x3 zero-pad conv (modules/model.py:109-110) run as four
        sub-pixel phases of a 2x2 conv on the un-upsampled input (2.25x fewer MACs; forward),
        and its adjoint as one 4x4 stride-2 conv over dy (data gradient)."""
        return (self.up == 2 and self.k == 3 and self.stride == 1 and self.pad_mode == DCS_PAD_ZERO
                and self.pads == (1, 1, 1, 1) and self.cout > 4 and self.cin % 16 == 0)

    # ---- weight packing ------------------------------------------------------------
    @property
    def win(self) -> bool:
        """f16x3 window kernel for this geometry (3x3 stride-1 pad-1, csrc/conv_win.hip): the packs
        also carry the pre-split fp16 planes (``_dcs_h3``); used where the call's image fits."""
        return (_WIN and _h3() and self.k == 3 and self.stride == 1 and self.up == 1
                and self.pads == (1, 1, 1, 1) and self.cin % 16 == 0 and self.cout % 128 == 0)

    def _attach_h3(self, wpack: torch.Tensor, w: torch.Tensor, flip: int) -> torch.Tensor:
        ncols = self.cin if flip else self.cout
        K = 9 * (self.cout if flip else self.cin)
        # data-gradient packs carry a tap-major copy behind the planes (the ring kernel's B)
        hi = torch.empty((2 if flip else 1) * ncols, K, device=w.device, dtype=torch.float16)
        lo = torch.empty((2 if flip else 1) * ncols, K, device=w.device, dtype=torch.float16)
        wexp = torch.empty(1, device=w.device, dtype=torch.int32)
        if _BATCH is not None:  # prepack: one batched launch pair for every pack of the step
            scratch = torch.empty(lib.RANGE_PARTS, device=w.device, dtype=torch.float32)
            _BATCH.add(w, h3=1, Cout=self.cout, Cin=self.cin, h3_flip=flip, h3_ncols=ncols, h3_hi=hi, h3_lo=lo,
                       h3_wexp=wexp, h3_scratch=scratch)
        else:
            scratch = workspace(lib.query("dcs_pack_weights_h3_scratch_size"), w.device)
            lib.call("dcs_pack_weights_h3", _p(w), self.cout, self.cin, flip, ncols, _p(hi), _p(lo), _p(scratch),
                     _p(wexp), _stream())
        wpack._dcs_h3 = (hi, lo, wexp)
        return wpack

    @property
    def subwin(self) -> bool:
        """Sub-pixel window kernel for this up-conv's forward (csrc/conv_subpix.hip): its pack carries
        the pre-split phase weights (_dcs_sp) next to the rows pass's kind-3 pack."""
        return _SUBWIN and _h3() and self.subpixel and self.cout % 64 == 0 and self.cin % 16 == 0

    @property
    def s2win(self) -> bool:
        """The window phase kernels for this stride-2 3x3 or 4x4 zero-pad-1 conv (the down-convs, the
        PatchGAN layers): forward over the source's parity classes, data gradient over dx's."""
        return (_SUBWIN and _S2WIN and _h3() and self.stride == 2 and self.k in (3, 4) and self.up == 1 and
                self.pads == (1, 1, 1, 1) and self.pad_mode == DCS_PAD_ZERO and self.cout % 128 == 0 and
                self.cin % 64 == 0)

    def _attach_sp(self, wpack: torch.Tensor, w: torch.Tensor, kind: int = 0) -> torch.Tensor:
        """Pre-split planes of the window phase kernels (dcs_pack_subpix_h3 kind: 0 / 1 sub-pixel forward /
        data gradient, 2 / 3 stride-2 data gradient / forward) on the pack as _dcs_sp."""
        shape = {0: (4 * self.cout, 4 * self.cin), 1: (self.cin, 16 * self.cout), 2: (4 * self.cin, 4 * self.cout),
                 3: (self.cout, 16 * self.cin), 4: (self.cout, 16 * self.cin), 5: (4 * self.cin, 4 * self.cout)}[kind]
        hi = torch.empty(*shape, device=w.device, dtype=torch.float16)
        lo = torch.empty_like(hi)
        wexp = torch.empty(1, device=w.device, dtype=torch.int32)
        scratch = torch.empty(lib.RANGE_PARTS, device=w.device, dtype=torch.float32)
        if _BATCH is not None:
            _BATCH.add(w, h3=2, Cout=self.cout, Cin=self.cin, h3_flip=kind, h3_hi=hi, h3_lo=lo, h3_wexp=wexp,
                       h3_scratch=scratch)
        else:
            lib.call("dcs_pack_subpix_h3", _p(w), self.cout, self.cin, kind, _p(hi), _p(lo), _p(scratch), _p(wexp),
                     _stream())
        wpack._dcs_sp = (hi, lo, wexp)
        return wpack

    def _key(self):
        return (self.cin, self.cout, self.k, self.stride, self.pads, self.pad_mode, self.up)

    def pack_fwd(self, w: torch.Tensor, cin_pad: Optional[int] = None) -> torch.Tensor:
        """B operand of the forward GEMM (cached per weight version, _cached_pack; recorded on the
        weight for prepack)."""
        _record_pack(w, "pack_fwd", self, cin_pad)
        return _cached_pack(w, ("fwd", self._key(), cin_pad), lambda: self._pack_fwd(w, cin_pad))

    def pack_dgrad(self, w: torch.Tensor, ci_count: Optional[int] = None) -> torch.Tensor:
        """B operand of the data-gradient GEMM (cached per weight version, _cached_pack; recorded on
        the weight for prepack)."""
        _record_pack(w, "pack_dgrad", self, ci_count)
        return _cached_pack(w, ("dgrad", self._key(), ci_count), lambda: self._pack_dgrad(w, ci_count))

    def _pack_fwd(self, w: torch.Tensor, cin_pad: Optional[int] = None) -> torch.Tensor:
        """B operand of the forward GEMM: N-major [Np][Kpad] for the MFMA rows pass (ldb =
        Kpad), K-major [K][1|4] for the narrow kernels (ldb = columns).  ``cin_pad``: the
        source carries that many channels (zero-padded beyond cin; the 4-channel stem)."""
        if cin_pad is not None and cin_pad != self.cin:
            return self._pack(w, 5, cin_pad, self.k * self.k * cin_pad, self.cout)
        if self.subpixel:
            out = self._pack(w, 3, self.cin, 16 * self.cin, self.cout)
            return self._attach_sp(out, w) if self.subwin else out
        K = self.k * self.k * self.cin
        out = self._pack(w, 0, self.cin, K, self.cout)
        if self.s2win:
            return self._attach_sp(out, w, 3 if self.k == 3 else 4)
        return self._attach_h3(out, w, 0) if self.win else out

    @property
    def c1_dgrad(self) -> bool:
        """One output channel, 'same' stride-1 padding (the Generator head): the data gradient runs
        on the VALU with the padding adjoint folded into the one-channel dy (dcs_conv_dgrad_c1)."""
        t, l, b, r = self.pads
        return (self.cout == 1 and self.cin in (32, 64) and self.k in (3, 7) and self.stride == 1 and self.up == 1
                and t == l == b == r and 2 * t == self.k - 1)

    def to1_dgrad(self, ci: int) -> bool:
        """Data gradient onto one input channel from 64 output channels (the image channel of the
        Generator stem, 7x7 reflect; the PatchGAN's first layer, 4x4 stride 2): two VALU passes,
        per-dy-pixel tap projections then a gather (dcs_conv_dgrad_to1)."""
        t, l, b, r = self.pads
        return (ci == 1 and self.cout == 64 and self.up == 1 and (self.k, self.stride) in ((7, 1), (4, 2))
                and (self.pad_mode == DCS_PAD_ZERO or (t == b and l == r)))

    def _pack_dgrad(self, w: torch.Tensor, ci_count: Optional[int] = None) -> torch.Tensor:
        ci = self.cin if ci_count is None else ci_count
        if self.c1_dgrad and ci == self.cin:  # forward K-major weights: [(ty*K+tx)*cin + c]
            return self._pack(w, 0, self.cin, self.k * self.k * self.cin, 1)
        if self.to1_dgrad(ci):  # un-flipped taps, K-major: [(ty*K+tx)*cout + co] = w[co][0][ty][tx]
            return self._pack(w, 2, 1, self.k * self.k * self.cout, 1)
        if self.subpixel and ci > 4:
            out = self._pack(w, 4, ci, 16 * self.cout, ci)
            return self._attach_sp(out, w, 1) if (self.subwin and _SUBWIN_D and ci == self.cin and ci % 128 == 0) else out
        kind = 2 if self.stride == 2 else 1
        K = self.k * self.k * self.cout
        out = self._pack(w, kind, ci, K, ci)
        if self.s2win and ci == self.cin:
            return self._attach_sp(out, w, 2 if self.k == 3 else 5)
        return self._attach_h3(out, w, 1) if (self.win and ci == self.cin) else out

    def _pack(self, w, kind, ci_count, K, ncols):
        if kind in (0, 1) and ncols > 4 and self.kslice:
            kind |= lib.PACK_KSLICE
        if ncols <= 4:
            Kpad, cols, nmajor = K, (1 if ncols == 1 else 4), 0
            out = torch.empty(Kpad, cols, device=w.device, dtype=torch.float32)
        else:
            Kpad, cols, nmajor = _round_up(K, 32), _round_up(ncols, _bn_for(ncols)), 1
            out = torch.empty(cols, Kpad, device=w.device, dtype=torch.float32)
        job = dict(Cout=self.cout, Cin=self.cin, KH=self.k, KW=self.k, kind=kind, ci_count=ci_count, Kpad=Kpad,
                   ncols=cols, nmajor=nmajor, out=out)
        if nmajor and _h3():  # f16x3 rows pass: the pack also writes the range record
            rng = torch.empty(lib.RANGE_PARTS, device=w.device, dtype=torch.float32)
            out._dcs_rng = (out._version, None, ACT_NONE, rng)
            planes = None
            if _BPRE and not self.win:  # pre-split fp16 planes for the rows pass (dcs_conv_desc.b_h3)
                planes = torch.empty(cols * 2 * Kpad, device=w.device, dtype=torch.float16)
                out._dcs_bh3 = (out._version, planes)
            if _BATCH is not None:
                _BATCH.add(w, rng=rng, planes=planes, **job)
            else:
                lib.call("dcs_pack_weights_r", _p(w), self.cout, self.cin, self.k, self.k, kind, ci_count, Kpad,
                         cols, nmajor, _p(out), _p(rng), _stream())
                if planes is not None:
                    lib.call("dcs_pack_split_h3", _p(out), cols, Kpad, _p(rng), lib.RANGE_PARTS, _p(planes),
                             _stream())
        elif _BATCH is not None:
            _BATCH.add(w, **job)
        else:
            lib.call("dcs_pack_weights", _p(w), self.cout, self.cin, self.k, self.k, kind, ci_count, Kpad,
                     cols, nmajor, _p(out), _stream())
        return out

    @staticmethod
    def _ldb(wpack: torch.Tensor, narrow: bool) -> int:
        return wpack.shape[1]  # Kpad (N-major) or columns (K-major): always the inner dim

    # ---- descriptors ---------------------------------------------------------------
    def _desc_fwd(self, s: Src, ldb: int, pro_act: int, epi_act: int, rows: bool = True) -> lib.ConvDesc:
        Ho, Wo = self.out_hw(s.H, s.W)
        d = lib.ConvDesc()
        d.N, d.Hs, d.Ws, d.Cs = s.N, s.H, s.W, s.C
        d.s_n, d.s_c, d.s_h, d.s_w = s.strides
        d.csplit = s.C if s.csplit is None else s.csplit
        d.s2_n, d.s2_c, d.s2_h, d.s2_w = s.strides2
        d.up, d.pad_mode = self.up, self.pad_mode
        d.KH = d.KW = self.k
        d.pt, d.pl = self.pads[0], self.pads[1]
        d.stride, d.parity = self.stride, 0
        if self.subpixel and rows:
            d.up, d.parity = 1, 2  # phases over the source grid (the upsample is in the weights)
        d.Ho, d.Wo, d.Co = Ho, Wo, self.cout
        d.ldb, d.pro_act, d.epi_act = ldb, pro_act, epi_act
        d.mma = _MMA if not _h3() else _fallback()  # f16x3 / f16: _set_mma with the ranges
        d.korder = lib.KORDER_SLICE if (rows and self.kslice and not self.narrow) else lib.KORDER_TAP
        return d

    # ---- forward -------------------------------------------------------------------
    def forward_in_stats(self, s: Src, wpack: torch.Tensor, bias: Optional[torch.Tensor] = None,
                         pro: Optional[Tuple[torch.Tensor, torch.Tensor, int]] = None,
                         epi_act: int = ACT_NONE, want_max: bool = False):
        """forward() and the InstanceNorm statistics of its output (the IN that follows every
        Generator / PatchGAN conv, modules/model.py:94-111, 124-129).  Where the rows pass applies
        (Ho*Wo % 128 == 0) the per-tile partials come out of the conv epilogue
        (dcs_conv_rows_in_stats) and one small kernel merges them (dcs_in_stats_finish): the
        statistics pass's re-read of the output is gone.  Otherwise: forward + in_stats."""
        Ho, Wo = self.out_hw(s.H, s.W)
        d = self._desc_fwd(s, wpack.shape[1], pro[2] if pro is not None else ACT_NONE, epi_act)
        nb = 0 if (self.narrow or not _FUSE_STATS) else lib.query("dcs_conv_rows_in_stats_parts_size", ctypes.byref(d))
        if nb and s.t2 is None:
            _set_mma(d, s.t, pro, _wrng(wpack), wpack)
        if nb and _STEM and bias is None and lib.query("dcs_stem_fwd_ok", ctypes.byref(d)):
            return self._stem(s, d, wpack, True, want_max)
        h3 = getattr(wpack, "_dcs_h3", None)
        if nb and h3 is not None and bias is None and lib.query("dcs_conv3_win_ok", ctypes.byref(d), 0):
            return self._win_in_stats(s, d, h3, nb, want_max)
        sp = getattr(wpack, "_dcs_sp", None)
        if nb and sp is not None and bias is None and s.t2 is None and self._phase_win_ok(d):
            return self._subpix(s, d, sp, True, want_max, pro)
        if nb == 0:
            out = self.forward(s, wpack, bias, pro, epi_act)
            return out, in_stats(out, want_max)
        assert s.C == self.cin or (s.C == 4 and self.cin < 4), (s.C, self.cin)
        _check_dev(s.t, s.t2, wpack, bias)
        dev = s.t.device
        out = torch.empty(s.N, Ho, Wo, self.cout, device=dev, dtype=torch.float32)
        parts = workspace(nb, dev)
        nchunk = ctypes.c_int(0)
        e0 = PROBE.begin() if _is_res_geom(self) else None
        lib.call("dcs_conv_rows_in_stats", ctypes.byref(d), _p(s.t), _p(s.t2), _p(wpack), _p(bias),
                 _p(pro[0]) if pro else None, _p(pro[1]) if pro else None, _p(out), _p(parts), parts.numel(),
                 ctypes.byref(nchunk), _stream())
        PROBE.end(e0, 2.0 * s.N * Ho * Wo * self.cout * self.cin * self.k * self.k)
        C = self.cout
        scale = torch.empty(s.N, C, device=dev, dtype=torch.float32)
        shift = torch.empty(s.N, C, device=dev, dtype=torch.float32)
        xmax = torch.empty(s.N, C, device=dev, dtype=torch.float32) if want_max else None
        xam = torch.empty(s.N, C, device=dev, dtype=torch.int32) if want_max else None
        lib.call("dcs_in_stats_finish", _p(parts), s.N, C, nchunk.value, IN_EPS, _p(scale), _p(shift), _p(xmax),
                 _p(xam), _stream())
        return out, INStats(scale, shift, xmax, xam)

    def _stem(self, s: Src, d, wpack, stats: bool, want_max: bool = False):
        """The Generator stem (7x7 reflect-pad-3, NHWC x 4 source -> 64) on its MFMA kernel
        (csrc/conv_stem.hip), with the IN statistics of its output when ``stats``."""
        dev = s.t.device
        d.mma = _fixed_mma("stem")
        out = torch.empty(s.N, s.H, s.W, self.cout, device=dev, dtype=torch.float32)
        parts = workspace(lib.query("dcs_stem_fwd_parts_size", ctypes.byref(d)), dev) if stats else None
        nchunk = ctypes.c_int(0)
        lib.call("dcs_stem_fwd", ctypes.byref(d), _p(s.t), _p(wpack), _p(out), _p(parts),
                 parts.numel() if stats else 0, ctypes.byref(nchunk), _stream())
        if not stats:
            return out
        C = self.cout
        scale = torch.empty(s.N, C, device=dev, dtype=torch.float32)
        shift = torch.empty(s.N, C, device=dev, dtype=torch.float32)
        xmax = torch.empty(s.N, C, device=dev, dtype=torch.float32) if want_max else None
        xam = torch.empty(s.N, C, device=dev, dtype=torch.int32) if want_max else None
        lib.call("dcs_in_stats_finish", _p(parts), s.N, C, nchunk.value, IN_EPS, _p(scale), _p(shift), _p(xmax),
                 _p(xam), _stream())
        return out, INStats(scale, shift, xmax, xam)

    def _phase_tag(self) -> Optional[str]:
        """The layer's key in _PHASE_F16X3: "up1" / "up2" (the up-convs 256->128, 128->64), "pg64" /
        "pg128" / "pg256" (the PatchGAN 4x4 layers by input channels); None for the down-convs."""
        if self.subpixel:
            return "up1" if self.cin >= 256 else "up2"
        return f"pg{self.cin}" if self.k == 4 else None

    def _phase_mma(self, d) -> None:
        """Operand mode of the window phase kernels' forward and data gradient: the step's mode, except
        the layers in _PHASE_F16X3, which take f16x3 in both fp16 modes as the stem and head do (in
        round 4 the up-convs and PatchGAN layers on fp16 missed the config-5 fixture's bar,
        profiles/r04ah; since round 6 they hold it)."""
        if self._phase_tag() in _PHASE_F16X3:
            d.mma = lib.MMA_F16X3

    def _phase_win_ok(self, d) -> bool:
        """d (a forward descriptor) is one the window phase kernels cover, in their operand mode."""
        mma = d.mma
        self._phase_mma(d)
        ok = lib.query("dcs_subpix_win_ok" if self.subpixel else "dcs_stride2_win_ok", ctypes.byref(d))
        d.mma = mma
        return bool(ok)

    def _subpix(self, s: Src, d, sp, stats: bool, want_max: bool = False, pro=None):
        """An up- or down-conv (or PatchGAN layer) forward (+ the IN statistics of its output when
        ``stats``) on the window phase kernels (csrc/conv_subpix.hip), operand mode as _phase_mma."""
        dev = s.t.device
        self._phase_mma(d)
        Ho, Wo = self.out_hw(s.H, s.W)
        out = torch.empty(s.N, Ho, Wo, self.cout, device=dev, dtype=torch.float32)
        api = "dcs_subpix_win" if self.subpixel else "dcs_stride2_win"
        parts = workspace(lib.query(api + "_parts_size", ctypes.byref(d)), dev) if stats else None
        nchunk = ctypes.c_int(0)
        pre = () if self.subpixel else (_p(pro[0]) if pro else None, _p(pro[1]) if pro else None)
        lib.call(api, ctypes.byref(d), _p(s.t), *pre, _p(sp[0]), _p(sp[1]), _p(sp[2]), _p(out), _p(parts),
                 parts.numel() if stats else 0, ctypes.byref(nchunk), _stream())
        if not stats:
            return out
        C = self.cout
        scale = torch.empty(s.N, C, device=dev, dtype=torch.float32)
        shift = torch.empty(s.N, C, device=dev, dtype=torch.float32)
        xmax = torch.empty(s.N, C, device=dev, dtype=torch.float32) if want_max else None
        xam = torch.empty(s.N, C, device=dev, dtype=torch.int32) if want_max else None
        lib.call("dcs_in_stats_finish", _p(parts), s.N, C, nchunk.value, IN_EPS, _p(scale), _p(shift), _p(xmax),
                 _p(xam), _stream())
        return out, INStats(scale, shift, xmax, xam)

    def _phase_win(self, d, dy: torch.Tensor, sp, out: torch.Tensor) -> bool:
        """An up- or down-conv (or PatchGAN layer) data gradient on the window phase kernels
        (csrc/conv_subpix.hip; operand mode as the forward, _phase_mma); False where the descriptor is not
        one they cover (the rows pass runs it)."""
        mma = d.mma
        self._phase_mma(d)
        if self.subpixel and lib.query("dcs_subpix_win_dgrad_ok", ctypes.byref(d)):
            lib.call("dcs_subpix_win_dgrad", ctypes.byref(d), _p(dy), _p(sp[0]), _p(sp[1]), _p(sp[2]), _p(out),
                     _stream())
            return True
        if self.stride == 2 and lib.query("dcs_stride2_win_ok", ctypes.byref(d)):
            lib.call("dcs_stride2_win", ctypes.byref(d), _p(dy), None, None, _p(sp[0]), _p(sp[1]), _p(sp[2]), _p(out),
                     None, 0, None, _stream())
            return True
        d.mma = mma
        return False

    def _win_in_stats(self, s: Src, d, h3, nb, want_max):
        """Forward + IN statistics on the f16x3 window kernel (csrc/conv_win.hip)."""
        dev = s.t.device
        Ho, Wo = self.out_hw(s.H, s.W)
        out = torch.empty(s.N, Ho, Wo, self.cout, device=dev, dtype=torch.float32)
        parts = workspace(nb, dev)
        nchunk = ctypes.c_int(0)
        e0 = PROBE.begin() if _is_res_geom(self) else None
        lib.call("dcs_conv3_win_in_stats", ctypes.byref(d), _p(s.t), _p(h3[0]), _p(h3[1]), _p(h3[2]), _p(out),
                 _p(parts), parts.numel(), ctypes.byref(nchunk), _stream())
        PROBE.end(e0, 2.0 * s.N * Ho * Wo * self.cout * self.cin * self.k * self.k)
        C = self.cout
        scale = torch.empty(s.N, C, device=dev, dtype=torch.float32)
        shift = torch.empty(s.N, C, device=dev, dtype=torch.float32)
        xmax = torch.empty(s.N, C, device=dev, dtype=torch.float32) if want_max else None
        xam = torch.empty(s.N, C, device=dev, dtype=torch.int32) if want_max else None
        lib.call("dcs_in_stats_finish", _p(parts), s.N, C, nchunk.value, IN_EPS, _p(scale), _p(shift), _p(xmax),
                 _p(xam), _stream())
        return out, INStats(scale, shift, xmax, xam)

    def forward(self, s: Src, wpack: torch.Tensor, bias: Optional[torch.Tensor] = None,
                pro: Optional[Tuple[torch.Tensor, torch.Tensor, int]] = None,
                epi_act: int = ACT_NONE, pro_max: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``pro_max``: per-(image, channel) max of the source before its prologue (INStats.xmax), for
        the Generator head's tap-projection kernel in the fp16 modes (csrc/conv_head.hip)."""
        assert s.C == self.cin or (s.C == 4 and self.cin < 4), (s.C, self.cin)
        _check_dev(s.t, s.t2, wpack, bias)
        Ho, Wo = self.out_hw(s.H, s.W)
        pro_act = pro[2] if pro is not None else ACT_NONE
        d = self._desc_fwd(s, wpack.shape[1], pro_act, epi_act)
        out = torch.empty(s.N, Ho, Wo, self.cout, device=s.t.device, dtype=torch.float32)
        if self.narrow and _HEAD_PROJ and pro is not None and pro_max is not None and _h3() and s.t2 is None:
            d.mma = _fixed_mma("head")
            if lib.query("dcs_head_fwd_proj_ok", ctypes.byref(d)):
                lib.call("dcs_head_fwd_proj", ctypes.byref(d), _p(s.t), _p(wpack), _p(bias), _p(pro[0]), _p(pro[1]),
                         _p(pro_max), _p(out), _stream())
                return out
            d.mma = _fallback()
        fn = "dcs_conv_rows_narrow" if self.narrow else "dcs_conv_rows"
        if not self.narrow and s.t2 is None:
            _set_mma(d, s.t, pro, _wrng(wpack), wpack)
            if _STEM and bias is None and lib.query("dcs_stem_fwd_ok", ctypes.byref(d)):
                return self._stem(s, d, wpack, False)
            sp = getattr(wpack, "_dcs_sp", None)
            if sp is not None and bias is None and self._phase_win_ok(d):
                return self._subpix(s, d, sp, False, pro=pro)
        h3 = getattr(wpack, "_dcs_h3", None)
        e0 = PROBE.begin() if _is_res_geom(self) else None
        if h3 is not None and bias is None and lib.query("dcs_conv3_win_ok", ctypes.byref(d), 0):
            lib.call("dcs_conv3_win_in_stats", ctypes.byref(d), _p(s.t), _p(h3[0]), _p(h3[1]), _p(h3[2]), _p(out),
                     None, 0, None, _stream())
        else:
            lib.call(fn, ctypes.byref(d), _p(s.t), _p(s.t2), _p(wpack), _p(bias),
                     _p(pro[0]) if pro else None, _p(pro[1]) if pro else None, _p(out), _stream())
        PROBE.end(e0, 2.0 * s.N * Ho * Wo * self.cout * self.cin * self.k * self.k)
        return out

    # ---- data gradient ---------------------------------------------------------------
    def dgrad(self, dy: torch.Tensor, wpack_d: torch.Tensor, H: int, W: int,
              ci_count: Optional[int] = None, addend: Optional[torch.Tensor] = None, inbwd=None):
        """dL/d(input) [N,H,W,ci] (NHWC) of this conv given dy [N,Ho,Wo,cout] (NHWC).  ``inbwd`` = (y,
        INStats, act) of the layer a = act(IN(y)) whose input gradient this is: where the window path
        applies, its partial sums are fused (dcs_conv_dgrad_reflect_win_inbwd) and the call returns
        (dx, parts, nchunk) for in_act_backward_parts, else (dx, None, 0)."""
        if inbwd is not None:
            r = self._dgrad_inbwd(dy, wpack_d, H, W, inbwd)
            if r is None:
                r = self._phase_dgrad_inbwd(dy, wpack_d, H, W, inbwd)
            if r is not None:
                return r
            return self.dgrad(dy, wpack_d, H, W, ci_count, addend), None, 0
        _check_dev(dy, wpack_d, addend)
        N, Ho, Wo, Co = dy.shape
        assert Co == self.cout
        ci = self.cin if ci_count is None else ci_count
        if self.c1_dgrad and ci == self.cin:
            out = torch.empty(N, H, W, ci, device=dy.device, dtype=torch.float32)
            lib.call("dcs_conv_dgrad_c1", _p(dy.contiguous()), N, H, W, _p(wpack_d), ci, self.k, self.pads[0],
                     self.pad_mode, _p(out), _stream())
            if addend is not None:
                lib.call("dcs_scale_add", _p(out), _p(addend), 1.0, out.numel(), _stream())
            return out
        if self.to1_dgrad(ci):
            out = torch.empty(N, H, W, 1, device=dy.device, dtype=torch.float32)
            dyc = dy.contiguous()
            ws = torch.empty(lib.query("dcs_conv_dgrad_to1_workspace_size", N, Ho, Wo, self.k) // 4,
                             device=dy.device, dtype=torch.float32)
            lib.call("dcs_conv_dgrad_to1", _p(dyc), N, Ho, Wo, Co, _p(wpack_d), self.k, self.stride,
                     self.pads[0], self.pads[1], self.pad_mode, H, W, _p(out), _p(ws), ws.numel() * 4, _stream())
            if addend is not None:
                lib.call("dcs_scale_add", _p(out), _p(addend), 1.0, out.numel(), _stream())
            return out
        narrow = ci <= 4
        fn = "dcs_conv_rows_narrow" if narrow else "dcs_conv_rows"
        d = lib.ConvDesc()
        d.N, d.Hs, d.Ws, d.Cs = N, Ho, Wo, Co
        d.s_n, d.s_c, d.s_h, d.s_w = Ho * Wo * Co, 1, Wo * Co, Co
        d.csplit = Co
        d.up, d.pad_mode = 1, DCS_PAD_ZERO
        d.KH = d.KW = self.k
        d.ldb, d.pro_act, d.epi_act = wpack_d.shape[1], ACT_NONE, ACT_NONE
        d.mma = _fallback() if _h3() else _MMA
        if not narrow:
            _set_mma(d, dy, None, _wrng(wpack_d), wpack_d)
        d.korder = lib.KORDER_SLICE if (self.kslice and ci > 4) else lib.KORDER_TAP
        d.Co = ci
        dev = dy.device
        t, l, b, r = self.pads
        if self.subpixel and not narrow:
            # adjoint of the sub-pixel forward: a 4x4 stride-2 pad-1 conv over dy (kind-4 pack)
            d.KH = d.KW = 4
            d.stride, d.parity, d.pt, d.pl = 2, 0, 1, 1
            d.Ho, d.Wo = H, W
            out = torch.empty(N, H, W, ci, device=dev, dtype=torch.float32)
            sp = getattr(wpack_d, "_dcs_sp", None)
            if sp is None or narrow or not self._phase_win(d, dy, sp, out):
                lib.call(fn, ctypes.byref(d), _p(dy), None, _p(wpack_d), None, None, None, _p(out), _stream())
            if addend is not None:
                lib.call("dcs_scale_add", _p(out), _p(addend), 1.0, out.numel(), _stream())
            return out
        if self.stride == 2:
            assert self.up == 1 and self.pad_mode == DCS_PAD_ZERO
            d.stride, d.parity, d.pt, d.pl = 2, 1, t, l
            d.Ho, d.Wo = H, W
            out = torch.empty(N, H, W, ci, device=dev, dtype=torch.float32)
            sp = getattr(wpack_d, "_dcs_sp", None)
            if sp is None or narrow or not self._phase_win(d, dy, sp, out):
                lib.call(fn, ctypes.byref(d), _p(dy), None, _p(wpack_d), None, None, None, _p(out),
                         _stream())
            if addend is not None:
                lib.call("dcs_scale_add", _p(out), _p(addend), 1.0, out.numel(), _stream())
            return out
        d.stride, d.parity = 1, 0
        Hv, Wv = H * self.up, W * self.up
        if self.pad_mode == DCS_PAD_REFLECT:
            assert self.up == 1 and t == b and l == r and t == l
            p = t
            d.pt = d.pl = self.k - 1
            d.Ho, d.Wo = Hv + 2 * p, Wv + 2 * p
            h3 = getattr(wpack_d, "_dcs_h3", None)
            if h3 is not None and not narrow and dy.is_contiguous() and \
                    lib.query("dcs_conv3_win_ok", ctypes.byref(d), 1):
                out = torch.empty(N, H, W, ci, device=dev, dtype=torch.float32)
                ring = torch.empty(lib.query("dcs_conv_dgrad_reflect_ring_size", ctypes.byref(d)) // 4,
                                   device=dev, dtype=torch.float32)
                e0 = PROBE.begin() if _is_res_geom(self) else None
                lib.call("dcs_conv_dgrad_reflect_win", ctypes.byref(d), _p(dy), _p(wpack_d), _p(h3[0]), _p(h3[1]),
                         _p(h3[2]), _p(addend), _p(out), _p(ring), _stream())
                PROBE.end(e0, 2.0 * N * H * W * self.cout * ci * self.k * self.k)
                return out
            if _FUSE_FOLD and addend is None and p == 1 and self.k == 3 and H >= 4 and W >= 4 and not narrow \
                    and dy.is_contiguous() and ci % 4 == 0:
                # interior written by the conv epilogue, the ring folded in after.  With a residual
                # addend the padded pass + dcs_reflect_fold stays faster: the addend read in the
                # epilogue sits after the MFMA loop (+145 us per 16-image launch against +125 us for
                # the whole fold pass, profiles/r02e_kernel_table.md)
                ring = lib.query("dcs_conv_dgrad_reflect_ring_size", ctypes.byref(d)) // 4
                buf = torch.empty(N * H * W * ci + ring, device=dev, dtype=torch.float32)
                out = buf[:N * H * W * ci].view(N, H, W, ci)
                e0 = PROBE.begin() if _is_res_geom(self) else None
                lib.call("dcs_conv_dgrad_reflect", ctypes.byref(d), _p(dy), _p(wpack_d), None, _p(out),
                         ctypes.c_void_p(buf.data_ptr() + N * H * W * ci * 4), _stream())
                PROBE.end(e0, 2.0 * N * Ho * Wo * self.cout * ci * self.k * self.k)
                return out
            dpad = torch.empty(N, d.Ho, d.Wo, ci, device=dev, dtype=torch.float32)
            e0 = PROBE.begin() if _is_res_geom(self) else None
            lib.call(fn, ctypes.byref(d), _p(dy), None, _p(wpack_d), None, None, None, _p(dpad), _stream())
            PROBE.end(e0, 2.0 * N * Ho * Wo * self.cout * ci * self.k * self.k)
            out = torch.empty(N, H, W, ci, device=dev, dtype=torch.float32)
            lib.call("dcs_reflect_fold", _p(dpad), _p(addend), _p(out), N, H, W, ci, p, _stream())
            return out
        d.pt, d.pl = self.k - 1 - t, self.k - 1 - l
        d.Ho, d.Wo = Hv, Wv
        dv = torch.empty(N, Hv, Wv, ci, device=dev, dtype=torch.float32)
        lib.call(fn, ctypes.byref(d), _p(dy), None, _p(wpack_d), None, None, None, _p(dv), _stream())
        if self.up == 2:
            out = torch.empty(N, H, W, ci, device=dev, dtype=torch.float32)
            lib.call("dcs_upsample2_grad", _p(dv), _p(out), N, H, W, ci, _stream())
        else:
            out = dv
        if addend is not None:
            lib.call("dcs_scale_add", _p(out), _p(addend), 1.0, out.numel(), _stream())
        return out

    def _phase_dgrad_inbwd(self, dy, wpack_d, H, W, inbwd):
        """The up- / down-conv data gradient on the window phase kernels with the IN-backward partial sums
        of its output fused (dcs_phase_win_dgrad_inbwd); None where they do not apply."""
        sp = getattr(wpack_d, "_dcs_sp", None)
        if sp is None or not dy.is_contiguous() or not (self.subpixel or self.stride == 2):
            return None
        N, Ho, Wo, Co = dy.shape
        d = lib.ConvDesc()
        d.N, d.Hs, d.Ws, d.Cs = N, Ho, Wo, Co
        d.s_n, d.s_c, d.s_h, d.s_w = Ho * Wo * Co, 1, Wo * Co, Co
        d.csplit = Co
        d.up, d.pad_mode = 1, DCS_PAD_ZERO
        d.ldb, d.pro_act, d.epi_act = wpack_d.shape[1], ACT_NONE, ACT_NONE
        d.mma = _fallback() if _h3() else _MMA
        _set_mma(d, dy, None, _wrng(wpack_d), wpack_d)
        d.korder = lib.KORDER_TAP
        d.Co = self.cin
        if self.subpixel:
            d.KH = d.KW = 4
            d.stride, d.parity, d.pt, d.pl = 2, 0, 1, 1
        else:
            d.KH = d.KW = self.k
            d.stride, d.parity, d.pt, d.pl = 2, 1, self.pads[0], self.pads[1]
        d.Ho, d.Wo = H, W
        self._phase_mma(d)
        sub = 1 if self.subpixel else 0
        nb = lib.query("dcs_phase_win_dgrad_inbwd_parts_size", ctypes.byref(d), sub)
        if nb == 0:
            return None
        y, st, act = inbwd
        out = torch.empty(N, H, W, self.cin, device=dy.device, dtype=torch.float32)
        parts = torch.empty(nb // 4, device=dy.device, dtype=torch.float32)
        nchunk = ctypes.c_int(0)
        lib.call("dcs_phase_win_dgrad_inbwd", ctypes.byref(d), sub, _p(dy), _p(sp[0]), _p(sp[1]), _p(sp[2]), _p(out),
                 _p(y), _p(st.scale), _p(st.shift), act, _p(parts), nb, ctypes.byref(nchunk), _stream())
        return out, parts, nchunk.value

    def _dgrad_inbwd(self, dy, wpack_d, H, W, inbwd):
        h3 = getattr(wpack_d, "_dcs_h3", None)
        if h3 is None or not dy.is_contiguous() or self.pad_mode != DCS_PAD_REFLECT or self.pads != (1, 1, 1, 1):
            return None
        N, Ho, Wo, Co = dy.shape
        d = lib.ConvDesc()
        d.N, d.Hs, d.Ws, d.Cs = N, Ho, Wo, Co
        d.s_n, d.s_c, d.s_h, d.s_w = Ho * Wo * Co, 1, Wo * Co, Co
        d.csplit = Co
        d.up, d.pad_mode = 1, DCS_PAD_ZERO
        d.KH = d.KW = self.k
        d.ldb, d.pro_act, d.epi_act = wpack_d.shape[1], ACT_NONE, ACT_NONE
        d.mma = _fallback() if _h3() else _MMA
        _set_mma(d, dy, None, _wrng(wpack_d))
        d.korder = lib.KORDER_SLICE if self.kslice else lib.KORDER_TAP
        d.Co = self.cin
        d.stride, d.parity = 1, 0
        d.pt = d.pl = self.k - 1
        d.Ho, d.Wo = H + 2, W + 2
        if not lib.query("dcs_conv3_win_ok", ctypes.byref(d), 1):
            return None
        nb = lib.query("dcs_conv_dgrad_reflect_win_inbwd_parts_size", ctypes.byref(d))
        if nb == 0:
            return None
        y, st, act = inbwd
        dev = dy.device
        out = torch.empty(N, H, W, self.cin, device=dev, dtype=torch.float32)
        ring = torch.empty(lib.query("dcs_conv_dgrad_reflect_ring_size", ctypes.byref(d)) // 4, device=dev,
                           dtype=torch.float32)
        parts = torch.empty(nb // 4, device=dev, dtype=torch.float32)
        nchunk = ctypes.c_int(0)
        e0 = PROBE.begin() if _is_res_geom(self) else None
        lib.call("dcs_conv_dgrad_reflect_win_inbwd", ctypes.byref(d), _p(dy), _p(wpack_d), _p(h3[0]), _p(h3[1]),
                 _p(h3[2]), _p(out), _p(ring), _p(y), _p(st.scale), _p(st.shift), act, _p(parts), nb,
                 ctypes.byref(nchunk), _stream())
        PROBE.end(e0, 2.0 * N * H * W * self.cout * self.cin * self.k * self.k)
        return out, parts, nchunk.value

    # ---- weight gradient ---------------------------------------------------------------
    def wgrad(self, dy: torch.Tensor, s: Src,
              pro: Optional[Tuple[torch.Tensor, torch.Tensor, int]] = None,
              out: Optional[torch.Tensor] = None, pro_max: Optional[torch.Tensor] = None) -> torch.Tensor:
        """dL/dW in torch's OIHW layout.  ``pro_max``: as in forward (the head's projection path)."""
        _check_dev(dy, s.t, s.t2)
        pro_act = pro[2] if pro is not None else ACT_NONE
        d = self._desc_fwd(s, 0, pro_act, ACT_NONE, rows=not self.narrow)
        if self.narrow and _HEAD_PROJ and pro is not None and pro_max is not None and _h3() and s.t2 is None \
                and dy.is_contiguous():
            m0, d.mma = d.mma, _fixed_mma("head")
            if lib.query("dcs_head_fwd_proj_ok", ctypes.byref(d)):
                if out is None:
                    out = torch.empty(self.cout, self.cin, self.k, self.k, device=dy.device, dtype=torch.float32)
                ws = workspace(lib.query("dcs_head_wgrad_proj_workspace_size", ctypes.byref(d)), dy.device)
                lib.call("dcs_head_wgrad_proj", ctypes.byref(d), _p(dy), _p(s.t), _p(pro[0]), _p(pro[1]),
                         _p(pro_max), _p(out), _p(ws), ws.numel(), _stream())
                return out
            d.mma = m0
        if not self.narrow and s.t2 is None and _h3() and s.t.is_contiguous():
            _set_mma(d, dy, None, range_rec(s.t, pro))  # (weight gradients in the step's mode)
        if s.C != self.cin:  # zero-padded source channels (4-channel stem): weights have cin
            d.cw = self.cin
        assert tuple(dy.shape) == (s.N, d.Ho, d.Wo, self.cout), (dy.shape, d.Ho, d.Wo)
        if out is None:
            out = torch.empty(self.cout, self.cin, self.k, self.k, device=dy.device,
                              dtype=torch.float32)
        if _STEM and pro is None and dy.is_contiguous() and lib.query("dcs_stem_wgrad_ok", ctypes.byref(d)):
            ws = workspace(lib.query("dcs_stem_wgrad_workspace_size", ctypes.byref(d)), dy.device)
            d.mma = _fixed_mma("stem_wgrad")
            lib.call("dcs_stem_wgrad", ctypes.byref(d), _p(dy), _p(s.t), _p(out), _p(ws), ws.numel(), _stream())
            return out
        if self.narrow:
            nb = lib.query("dcs_conv_wgrad_narrow_workspace_size", ctypes.byref(d))
            ws = workspace(nb, dy.device)
            lib.call("dcs_conv_wgrad_narrow", ctypes.byref(d), _p(dy), _p(s.t), _p(s.t2),
                     _p(pro[0]) if pro else None, _p(pro[1]) if pro else None, _p(out), _p(ws),
                     ws.numel(), _stream())
        else:
            nb = lib.query("dcs_conv_wgrad_workspace_size", ctypes.byref(d))
            ws = workspace(nb, dy.device)
            lib.call("dcs_conv_wgrad", ctypes.byref(d), _p(dy), _p(s.t), _p(s.t2),
                     _p(pro[0]) if pro else None, _p(pro[1]) if pro else None, _p(out), _p(ws),
                     ws.numel(), _stream())
        return out


# ---------------------------------------------------------------------------------------
# InstanceNorm
# ---------------------------------------------------------------------------------------
class INStats:
    __slots__ = ("scale", "shift", "xmax", "xargmax")

    def __init__(self, scale, shift, xmax=None, xargmax=None):
        self.scale, self.shift, self.xmax, self.xargmax = scale, shift, xmax, xargmax


def pack_nhwc4(x: torch.Tensor, x2: Optional[torch.Tensor] = None) -> torch.Tensor:
    """NCHW image [N,c1,H,W] (+ NCHW masks [N,c2,H,W]) -> NHWC [N,H,W,4], zero channels after
    c1+c2: the layout of the vectorised stem gather (the trainer.py:451 concat, fused)."""
    x = x.contiguous()
    x2 = x2.contiguous() if x2 is not None else None
    _check_dev(x, x2)
    N, c1, H, W = x.shape
    c2 = x2.shape[1] if x2 is not None else 0
    out = torch.empty(N, H, W, 4, device=x.device, dtype=torch.float32)
    lib.call("dcs_pack_nhwc4", _p(x), c1, _p(x2), c2, N, H, W, _p(out), _out_rng(out), _stream())
    return out


def in_stats(x: torch.Tensor, want_max: bool = False) -> INStats:
    _check_dev(x)
    N, H, W, C = x.shape
    dev = x.device
    scale = torch.empty(N, C, device=dev, dtype=torch.float32)
    shift = torch.empty(N, C, device=dev, dtype=torch.float32)
    xmax = torch.empty(N, C, device=dev, dtype=torch.float32) if want_max else None
    xam = torch.empty(N, C, device=dev, dtype=torch.int32) if want_max else None
    nb = lib.query("dcs_in_stats_workspace_size", N, H * W, C)
    ws = workspace(nb, dev)
    lib.call("dcs_in_stats", _p(x), N, H * W, C, IN_EPS, _p(scale), _p(shift), _p(xmax), _p(xam),
             _p(ws), ws.numel(), _stream())
    return INStats(scale, shift, xmax, xam)


def in_apply(x: torch.Tensor, st: INStats, act: int) -> torch.Tensor:
    N, H, W, C = x.shape
    out = torch.empty_like(x)
    lib.call("dcs_in_apply", _p(x), _p(st.scale), _p(st.shift), _p(out), N, H * W, C, act, _out_rng(out), _stream())
    return out


def in_act_backward(da: torch.Tensor, y: torch.Tensor, st: INStats, act: int) -> torch.Tensor:
    N, H, W, C = y.shape
    dy = torch.empty_like(y)
    nb = lib.query("dcs_in_stats_workspace_size", N, H * W, C)
    ws = workspace(nb, y.device)
    lib.call("dcs_in_act_backward", _p(da), _p(y), _p(st.scale), _p(st.shift), _p(dy), N, H * W, C,
             act, _p(ws), ws.numel(), _out_rng(dy), _stream())
    return dy


def head_dgrad_in(dy_out: torch.Tensor, wk: torch.Tensor, y: torch.Tensor, st: INStats, act: int) -> Optional[torch.Tensor]:
    """in_act_backward(head.dgrad(dy_out), y, st, act) for the Generator head (7x7 reflect-pad-3
    64 -> 1) in the fp16 operand modes, with the 64-channel data gradient recomputed on MFMA inside
    the IN backward's two passes (dcs_head_dgrad_in).  ``wk``: the head's dgrad pack (K-major
    [49 * 64][1]).  None where it does not apply (other modes, act, or images below 8 x 8)."""
    N, H, W, C = y.shape
    if not (_HEAD_PROJ and _h3() and C == 64 and act == ACT_RELU and H >= 8 and W >= 8 and y.is_contiguous()
            and dy_out.numel() == N * H * W and wk.numel() == 49 * 64):
        return None
    _check_dev(dy_out, wk, y)
    dy = torch.empty_like(y)
    ws = workspace(lib.query("dcs_head_dgrad_in_workspace_size", N, H, W), y.device)
    g = dy_out.contiguous()
    g_rng = range_rec(g.view(N, H, W, 1))
    lib.call("dcs_head_dgrad_in", _p(g), _p(g_rng), g_rng.numel(), _p(wk), N, H, W, _p(y), _p(st.scale), _p(st.shift),
             act, _fixed_mma("head"), _p(dy), _p(ws), ws.numel(), _out_rng(dy), _stream())
    return dy


def in_act_backward_parts(da: torch.Tensor, y: torch.Tensor, st: INStats, act: int, parts: torch.Tensor,
                          nchunk: int) -> torch.Tensor:
    """in_act_backward with the partial sums its producer wrote (ConvGeom.dgrad(..., inbwd=...))."""
    N, H, W, C = y.shape
    dy = torch.empty_like(y)
    ws = workspace(N * C * 8, y.device)
    lib.call("dcs_in_act_backward_parts", _p(da), _p(y), _p(st.scale), _p(st.shift), _p(dy), N, H * W, C, act,
             _p(parts), nchunk, _p(ws), ws.numel(), _out_rng(dy), _stream())
    return dy


def act_backward(da: torch.Tensor, y: torch.Tensor, act: int) -> torch.Tensor:
    out = torch.empty_like(y)
    lib.call("dcs_act_backward", _p(da.contiguous()), _p(y), _p(out), y.numel(), act, _out_rng(out), _stream())
    return out


def channel_sum(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    C = x.shape[-1]
    Pn = x.numel() // C
    if out is None:
        out = torch.empty(C, device=x.device, dtype=torch.float32)
    assert out.numel() == C and out.is_contiguous()
    ws = workspace(lib.query("dcs_channel_sum_workspace_size", Pn, C), x.device)
    lib.call("dcs_channel_sum", _p(x), Pn, C, _p(out), _p(ws), ws.numel(), _stream())
    return out


def scale_add_(y: torch.Tensor, x: torch.Tensor, a: float = 1.0) -> torch.Tensor:
    assert y.numel() == x.numel() and y.is_contiguous() and x.is_contiguous()
    _drop_rng(y)
    lib.call("dcs_scale_add", _p(y), _p(x), float(a), y.numel(), _stream())
    return y


def scale_dev(x: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    out = torch.empty_like(x)
    lib.call("dcs_scale_dev", _p(x), _p(s), _p(out), x.numel(), _stream())
    return out


# ---------------------------------------------------------------------------------------
# CBAM
# ---------------------------------------------------------------------------------------
def cbam_forward(x, y, st: INStats, w1, w2, wsa):
    N, H, W, C = y.shape
    Cr = w1.shape[0]
    ksa = wsa.shape[-1]
    dev = y.device
    ca = torch.empty(N, C, device=dev, dtype=torch.float32)
    sin_ = torch.empty(N, H * W, 2, device=dev, dtype=torch.float32)
    sarg = torch.empty(N, H * W, device=dev, dtype=torch.int32)
    sa = torch.empty(N, H * W, device=dev, dtype=torch.float32)
    out = torch.empty_like(x)
    lib.call("dcs_cbam_forward", _p(x), _p(y), _p(st.scale), _p(st.shift), _p(st.xmax), _p(w1),
             _p(w2), _p(wsa), N, H, W, C, Cr, ksa, _p(ca), _p(sin_), _p(sarg), _p(sa), _p(out),
             _out_rng(out), _stream())
    return out, (ca, sin_, sarg, sa)


def cbam_backward(dout, y, st: INStats, w1, w2, wsa, saved, out_dw=(None, None, None)):
    """``out_dw``: optional destinations of (dw1, dw2, dwsa) shaped like w1 / w2 / wsa."""
    ca, sin_, sarg, sa = saved
    N, H, W, C = y.shape
    Cr = w1.shape[0]
    ksa = wsa.shape[-1]
    dy = torch.empty_like(y)
    dw1 = torch.empty_like(w1) if out_dw[0] is None else out_dw[0]
    dw2 = torch.empty_like(w2) if out_dw[1] is None else out_dw[1]
    dwsa = torch.empty_like(wsa) if out_dw[2] is None else out_dw[2]
    for o, ref in ((dw1, w1), (dw2, w2), (dwsa, wsa)):
        assert o.shape == ref.shape and o.is_contiguous()
    nb = lib.query("dcs_cbam_backward_workspace_size", N, H, W, C, Cr, ksa)
    ws = workspace(nb, y.device)
    lib.call("dcs_cbam_backward", _p(dout), _p(y), _p(st.scale), _p(st.shift), _p(st.xmax),
             _p(st.xargmax), _p(w1), _p(w2), _p(wsa), _p(ca), _p(sin_), _p(sarg), _p(sa), N, H, W,
             C, Cr, ksa, _p(dy), _p(dw1), _p(dw2), _p(dwsa), _p(ws), ws.numel(), _out_rng(dy), _stream())
    return dy, dw1, dw2, dwsa


# ---------------------------------------------------------------------------------------
# losses: value (0-d tensor) and d value / d pred
# ---------------------------------------------------------------------------------------
def _plane_dims(t):
    N, C, H, W = t.shape
    assert C == 1, "losses operate on single-channel planes"
    return N, H, W


def _loss_call(name, pred, args, want_grad):
    _check_dev(pred)
    N, H, W = _plane_dims(pred)
    dev = pred.device
    out = torch.empty(1, device=dev, dtype=torch.float32)
    grad = torch.empty_like(pred) if want_grad else None
    ws = workspace(lib.query("dcs_loss_workspace_size", N, H, W), dev)
    lib.call(name, *args(N, H, W), _p(out), _p(grad), _p(ws), ws.numel(), _stream())
    return out.view(()), grad


def loss_l1(pred, target, want_grad=True):
    p, t = pred.contiguous(), target.contiguous()
    return _loss_call("dcs_loss_l1", p, lambda N, H, W: (_p(p), _p(t), p.numel()), want_grad)


def loss_mse(pred, target, want_grad=True):
    p, t = pred.contiguous(), target.contiguous()
    return _loss_call("dcs_loss_mse", p, lambda N, H, W: (_p(p), _p(t), p.numel()), want_grad)


def loss_mse_const(pred, value: float, want_grad=True):
    p = pred.contiguous()
    return _loss_call("dcs_loss_mse_const", p, lambda N, H, W: (_p(p), float(value), p.numel()),
                      want_grad)


def loss_gradient(pred, target, want_grad=True):
    p, t = pred.contiguous(), target.contiguous()
    return _loss_call("dcs_loss_gradient", p, lambda N, H, W: (_p(p), _p(t), N, H, W), want_grad)


def loss_contrast_attention(pred, target, source, sigma, min_w, max_w, k, want_grad=True):
    p, t, s = pred.contiguous(), target.contiguous(), source.contiguous()
    return _loss_call("dcs_loss_contrast_attention", p,
                      lambda N, H, W: (_p(p), _p(t), _p(s), N, H, W, float(sigma), float(min_w),
                                       float(max_w), int(k)), want_grad)


def loss_contrast_region(pred, target, source, threshold, weight, want_grad=True):
    p, t, s = pred.contiguous(), target.contiguous(), source.contiguous()
    return _loss_call("dcs_loss_contrast_region", p,
                      lambda N, H, W: (_p(p), _p(t), _p(s), N, H, W, float(threshold),
                                       float(weight)), want_grad)


def loss_contrast_edge(pred, target, want_grad=True):
    p, t = pred.contiguous(), target.contiguous()
    return _loss_call("dcs_loss_contrast_edge", p, lambda N, H, W: (_p(p), _p(t), N, H, W),
                      want_grad)


def loss_contrast_region_global(pred, target, source, threshold, weight, allreduce, grad_scale, want_grad=True):
    """ContrastRegionLoss of the WHOLE data-parallel batch (SURVEY.md §8e option ii): this
    shard's partial sums, ``allreduce`` (in-place sum over ranks), then the whole-batch value
    and this shard's gradient times ``grad_scale``.  With an identity ``allreduce`` and
    grad_scale 1 it equals loss_contrast_region."""
    p, t, s = pred.contiguous(), target.contiguous(), source.contiguous()
    _check_dev(p, t, s)
    N, H, W = _plane_dims(p)
    dev = p.device
    ws = workspace(lib.query("dcs_loss_workspace_size", N, H, W), dev)  # one buffer for both phases
    red = torch.zeros(8, device=dev, dtype=torch.float64)
    lib.call("dcs_loss_contrast_region_partial", _p(p), _p(t), _p(s), N, H, W, float(threshold), _p(red), _p(ws),
             ws.numel(), _stream())
    allreduce(red)
    out = torch.empty(1, device=dev, dtype=torch.float32)
    grad = torch.empty_like(p) if want_grad else None
    lib.call("dcs_loss_contrast_region_finish", _p(p), N, H, W, float(weight), _p(red), float(grad_scale), _p(out),
             _p(grad), _p(ws), ws.numel(), _stream())
    return out.view(()), grad


def loss_contrast_edge_global(pred, target, allreduce, grad_scale, want_grad=True):
    """ContrastEdgeLoss of the WHOLE data-parallel batch: Sobel-magnitude mean/std and the exact
    top-10 % mean by a radix select whose four 256-bin histograms are summed over ranks.  Six
    small all-reduces per evaluation; no host synchronisation."""
    p, t = pred.contiguous(), target.contiguous()
    _check_dev(p, t)
    N, H, W = _plane_dims(p)
    dev = p.device
    ws = workspace(lib.query("dcs_loss_workspace_size", N, H, W), dev)
    red = torch.zeros(9, device=dev, dtype=torch.float64)
    hist = torch.empty(512, device=dev, dtype=torch.int32)
    lib.call("dcs_loss_contrast_edge_partial", _p(p), _p(t), N, H, W, _p(red), _p(ws), ws.numel(), _stream())
    allreduce(red[:5])
    for ps in range(4):
        lib.call("dcs_loss_contrast_edge_hist", N, H, W, ps, _p(red), _p(hist), _p(ws), ws.numel(), _stream())
        allreduce(hist)
        lib.call("dcs_loss_contrast_edge_select", ps, _p(hist), _p(ws), ws.numel(), _stream())
    lib.call("dcs_loss_contrast_edge_topk", N, H, W, _p(red), _p(ws), ws.numel(), _stream())
    allreduce(red[5:9])
    out = torch.empty(1, device=dev, dtype=torch.float32)
    grad = torch.empty_like(p) if want_grad else None
    lib.call("dcs_loss_contrast_edge_finish", _p(p), N, H, W, _p(red), float(grad_scale), _p(out), _p(grad), _p(ws),
             ws.numel(), _stream())
    return out.view(()), grad


def loss_ssim(X, Y, data_range=1.0, win=11, sigma=1.5, K=(0.01, 0.03), want_grad=True):
    x, y = X.contiguous(), Y.contiguous()
    return _loss_call("dcs_loss_ssim", x,
                      lambda N, H, W: (_p(x), _p(y), N, H, W, float(data_range), int(win),
                                       float(sigma), float(K[0]), float(K[1])), want_grad)


def gen_loss_fused(jobs, recipe=None, extra=(), ssim_data_range=1.0, ca=(0.15, 1.0, 3.0)):
    """The fused G-step loss kernel (include/ducosy_hip.h dcs_gen_loss_fused).

    jobs: dicts with pred [n,1,H,W] (contiguous), and as needed target, source, grad (written with
    the weighted sum of the selected terms' d/dpred), flags (lib.GL_*), c_l1 / c_grad / c_ssim /
    c_ca / c_mse coefficients, t_const, add0 / add1 with c_add0 / c_add1.
    recipe: (bias [nout], coef [nout][5 * len(jobs)], coefx [nout][4]) composing the outputs from
    the job terms' means (val[5 j + q]: q = 0 L1, 1 / 2 gradient-loss x / y, 3 SSIM, 4 CA or MSE)
    and up to four device scalars ``extra``.  Returns the [nout] output tensor (or None)."""
    arr = (lib.GLJob * len(jobs))()
    dev = jobs[0]["pred"].device
    for k, j in enumerate(jobs):
        p = j["pred"]
        _check_dev(p)
        assert p.is_contiguous() and p.dim() == 4 and p.shape[1] == 1, "loss planes: contiguous [n,1,H,W]"
        for key in ("target", "source", "grad", "add0", "add1"):
            t = j.get(key)
            if t is not None:
                assert t.is_contiguous() and t.shape == p.shape, key
        a = arr[k]
        a.pred, a.target, a.source = p.data_ptr(), _ptr(j.get("target")), _ptr(j.get("source"))
        a.add0, a.add1, a.grad = _ptr(j.get("add0")), _ptr(j.get("add1")), _ptr(j.get("grad"))
        a.n_img, a.H, a.W, a.flags = p.shape[0], p.shape[2], p.shape[3], int(j["flags"])
        for key in ("c_l1", "c_grad", "c_ssim", "c_ca", "c_mse", "t_const", "c_add0", "c_add1"):
            setattr(a, key, float(j.get(key, 0.0)))
    ws = workspace(lib.query("dcs_gen_loss_fused_ws", arr, len(jobs)), dev)
    out, nout = None, 0
    bias = coef = coefx = ex = None
    if recipe is not None:
        b, c, cx = recipe
        nout = len(b)
        bias = (ctypes.c_float * nout)(*b)
        coef = (ctypes.c_float * (nout * 5 * len(jobs)))(*[float(v) for row in c for v in row])
        coefx = (ctypes.c_float * (nout * 4))(*[float(v) for row in cx for v in row])
        ex = (ctypes.c_void_p * 4)(*[_ptr(e) for e in (list(extra) + [None] * 4)[:4]])
        out = torch.empty(nout, device=dev, dtype=torch.float32)
    lib.call("dcs_gen_loss_fused", arr, len(jobs), float(ssim_data_range), float(ca[0]), float(ca[1]), float(ca[2]),
             bias, coef, coefx, ex, nout, _p(out), _p(ws), ws.numel(), _stream())
    return out


def multi_add(pairs) -> None:
    """dst += src for a list of (src, dst) float32 tensors of equal numel, one launch per 64."""
    if not pairs:
        return
    n = len(pairs)
    src = (ctypes.c_void_p * n)(*[s.data_ptr() for s, _ in pairs])
    dst = (ctypes.c_void_p * n)(*[d.data_ptr() for _, d in pairs])
    cnt = (ctypes.c_int64 * n)(*[d.numel() for _, d in pairs])
    for s_, d_ in pairs:
        assert s_.numel() == d_.numel() and s_.is_contiguous() and d_.is_contiguous() and d_.dtype == torch.float32
    lib.call("dcs_multi_add", n, src, dst, cnt, _stream())


# ---------------------------------------------------------------------------------------
# optimizer
# ---------------------------------------------------------------------------------------
def adam_step(p, g, m, v, lr, beta1, beta2, eps, step):
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    lib.call("dcs_adam_step", _p(p), _p(g), _p(m), _p(v), p.numel(), float(lr), float(beta1),
             float(beta2), float(eps), float(bc1), float(bc2), _stream())


# ---------------------------------------------------------------------------------------
# input pipeline: HU transform + anatomical masks (modules/preprocess.py, mask_generator.py)
# ---------------------------------------------------------------------------------------
_RAW_DTYPES = {torch.int16: 0, torch.uint16: 1, torch.float32: 2} if hasattr(torch, "uint16") \
    else {torch.int16: 0, torch.float32: 2}
MASK_KINDS = ("lung", "mediastinum", "bone", "lung_vessel")
# mask_generator.py defaults: detect_lung(-1000, -300, min_size 64, border 32),
# detect_lung_vessels(-300, 600), detect_mediastinum(-300, 450), detect_bone(200, 0.25)
MASK_DEFAULTS = dict(lung_lower=-1000, lung_upper=-300, min_size=64, border_margin=32,
                     vessel_lower=-300, vessel_upper=600, mediastinum_lower=-300, mediastinum_upper=450,
                     bone_threshold=200, spine_margin_ratio=0.25)


def hu_transform(raw: torch.Tensor, slope: torch.Tensor, intercept: torch.Tensor, hu_min: float, hu_max: float,
                 soft: bool = True, sigma: float = 50.0, want_hu: bool = True, want_img: bool = True):
    """[N,H,W] stored pixels (int16/uint16/float32) -> (hu, img) float32 [N,H,W] on the device
    (preprocess.py:43-55 with apply_soft_squeezing :6-40).  slope/intercept: float32 [N]."""
    if not raw.is_cuda or not slope.is_cuda or not intercept.is_cuda:
        raise RuntimeError("ducosy HIP ops require device tensors (no CPU fallback)")
    if raw.dtype not in _RAW_DTYPES:
        raise RuntimeError(f"hu_transform: unsupported pixel dtype {raw.dtype}")
    if raw.dim() == 2:
        raw = raw[None]
    raw = raw.contiguous()
    N, H, W = raw.shape
    slope = slope.to(torch.float32).reshape(-1).contiguous()
    intercept = intercept.to(torch.float32).reshape(-1).contiguous()
    if slope.numel() != N or intercept.numel() != N:
        raise ValueError("hu_transform: one slope/intercept per slice")
    hu = torch.empty(N, H, W, device=raw.device, dtype=torch.float32) if want_hu else None
    img = torch.empty(N, H, W, device=raw.device, dtype=torch.float32) if want_img else None
    lib.call("dcs_hu_transform", _p(raw), _RAW_DTYPES[raw.dtype], _p(slope), _p(intercept), N, H, W,
             float(hu_min), float(hu_max), int(bool(soft)), float(sigma), _p(hu), _p(img), _stream())
    return hu, img


def anatomical_masks(hu: torch.Tensor, mask_types=MASK_KINDS, out: Optional[torch.Tensor] = None,
                     lung_mask: Optional[torch.Tensor] = None, **params):
    """HU slices [N,H,W] float32 -> float32 masks [N, len(mask_types), H, W] in mask_types order
    (generate_anatomical_masks per 2-D slice + the channel concat of dataset.py:135-158).
    lung_mask (optional, binary [N,H,W]) replaces detect_lung, as the lung_mask argument of
    detect_mediastinum / detect_bone / detect_lung_vessels."""
    _check_dev(hu, lung_mask)
    if hu.dtype != torch.float32:
        raise RuntimeError("anatomical_masks: HU must be float32")
    if hu.dim() == 2:
        hu = hu[None]
    hu = hu.contiguous()
    N, H, W = hu.shape
    kinds = list(mask_types)
    if not kinds or any(k not in MASK_KINDS for k in kinds) or len(set(kinds)) != len(kinds):
        raise ValueError(f"anatomical_masks: mask_types must be distinct names from {MASK_KINDS}")
    p = dict(MASK_DEFAULTS)
    unknown = set(params) - set(p)
    if unknown:
        raise TypeError(f"anatomical_masks: unknown parameters {sorted(unknown)}")
    p.update(params)
    nout = len(kinds)
    if out is None:
        out = torch.empty(N, nout, H, W, device=hu.device, dtype=torch.float32)
    elif out.shape != (N, nout, H, W) or not out.is_contiguous() or out.dtype != torch.float32:
        raise ValueError("anatomical_masks: out must be a contiguous float32 [N, nout, H, W] tensor")
    thr = (ctypes.c_float * 7)(p["lung_lower"], p["lung_upper"], p["vessel_lower"], p["vessel_upper"],
                               p["mediastinum_lower"], p["mediastinum_upper"], p["bone_threshold"])
    # spine_start = int(height * (1 - spine_margin_ratio))  (mask_generator.py:212)
    ip = (ctypes.c_int32 * 3)(int(p["min_size"]), int(p["border_margin"]),
                              int(H * (1 - p["spine_margin_ratio"])))
    ch = (ctypes.c_int32 * 4)(*[kinds.index(k) if k in kinds else -1 for k in MASK_KINDS])
    lung_in = None
    if lung_mask is not None:
        lung_in = (lung_mask.reshape(N, H, W) != 0).to(torch.uint8).contiguous()
    nb = lib.query("dcs_masks_workspace_size", N, H, W)
    ws = workspace(nb, hu.device)
    lib.call("dcs_anatomical_masks", _p(hu), _p(lung_in), N, H, W, thr, ip, ch, nout, _p(out), _p(ws), ws.numel(),
             _stream())
    return out
