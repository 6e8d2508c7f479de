"""Adam over one flat parameter buffer (torch.optim.Adam semantics, modules/trainer.py:360-362).

Parameters, gradients and both moments are re-bound as views of four flat device buffers,
so the whole optimizer step is ONE HIP kernel launch and the data-parallel gradient
all-reduce is ONE collective per optimizer.  ``state_dict()`` / ``load_state_dict()`` keep
torch.optim.Adam's layout (per-parameter ``step`` / ``exp_avg`` / ``exp_avg_sq``, same
param_groups keys), so checkpoints interoperate with the reference.
"""
from __future__ import annotations

import torch

from .hip import ops


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        params = list(params)
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=0, amsgrad=False, maximize=False,
                        foreach=None, capturable=False, differentiable=False, fused=None,
                        decoupled_weight_decay=False)
        super().__init__(params, defaults)
        if len(self.param_groups) != 1:
            raise ValueError("FusedAdam: one parameter group")
        plist = self.param_groups[0]["params"]
        dev = plist[0].device
        if dev.type != "cuda":
            raise RuntimeError("FusedAdam runs on the HIP kernels: move the model to the GPU first")
        total = sum(p.numel() for p in plist)
        self.flat_p = torch.empty(total, device=dev, dtype=torch.float32)
        self.flat_g = torch.zeros(total, device=dev, dtype=torch.float32)
        self.flat_m = torch.zeros(total, device=dev, dtype=torch.float32)
        self.flat_v = torch.zeros(total, device=dev, dtype=torch.float32)
        off = 0
        for p in plist:
            n = p.numel()
            self.flat_p[off:off + n].copy_(p.detach().reshape(-1))
            p.data = self.flat_p[off:off + n].view_as(p)
            p.grad = self.flat_g[off:off + n].view_as(p)
            self.state[p] = {"step": torch.tensor(0.0),
                             "exp_avg": self.flat_m[off:off + n].view_as(p),
                             "exp_avg_sq": self.flat_v[off:off + n].view_as(p)}
            off += n
        self._t = 0

    def zero_grad(self, set_to_none: bool = True):
        """Zero the flat gradient buffer (the per-parameter grads stay views of it).  Each parameter is
        marked fresh with a stamp (storage address, version counter) of its zeroed .grad: the fused
        networks' backward (modules/hip/networks.py _GradSink) writes its first gradient straight into
        that .grad instead of handing it to AccumulateGrad, but only while the stamp still matches.
        Any torch in-place write to the flat buffer (AccumulateGrad's add of an ordinary autograd
        contribution, a user regulariser) bumps the version counter the views share, and a replaced
        .grad changes the address: the parameter is then no longer fresh and its fused contribution
        is added, not written over."""
        self.flat_g.zero_()
        v = self.flat_g._version
        for p in self.param_groups[0]["params"]:
            p._dcs_fresh = (p.grad.data_ptr(), v) if p.grad is not None else None

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        g = self.param_groups[0]
        self._t += 1
        b1, b2 = g["betas"]
        ops.adam_step(self.flat_p, self.flat_g, self.flat_m, self.flat_v, g["lr"], b1, b2, g["eps"], self._t)
        ops.bump_weights_epoch(g["params"])  # the kernel wrote them behind autograd's version counter
        return loss

    def state_dict(self):
        for p in self.param_groups[0]["params"]:
            self.state[p]["step"] = torch.tensor(float(self._t))
        sd = super().state_dict()
        sd["state"] = {k: {kk: (vv.clone() if torch.is_tensor(vv) else vv) for kk, vv in v.items()}
                       for k, v in sd["state"].items()}
        return sd

    def load_state_dict(self, state_dict):
        views = {p: (self.state[p]["exp_avg"], self.state[p]["exp_avg_sq"])
                 for p in self.param_groups[0]["params"]}
        super().load_state_dict(state_dict)
        t = 0
        for p, (m, v) in views.items():
            st = self.state.get(p, {})
            if "exp_avg" in st:
                m.copy_(st["exp_avg"].reshape(m.shape))
                v.copy_(st["exp_avg_sq"].reshape(v.shape))
                t = max(t, int(float(st["step"])))
            self.state[p] = {"step": torch.tensor(float(t)), "exp_avg": m, "exp_avg_sq": v}
        self._t = t
