"""Deterministic, platform-independent parameter/input generator for tests.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import anything under ``oracle/``.

A splitmix64 counter stream (pure numpy uint64 arithmetic) so that the golden
fixture script (run once in the build container against the reference) and the
parity tests (run here and on the GPU box) regenerate bit-identical weights and
inputs without storing megabytes of parameters in ``tests/golden/``.

Initialisation follows the reference's semantics:
  * conv weights ~ N(0, 0.02)                      (modules/model.py:134-137)
  * conv biases  ~ U(-1/sqrt(fan_in), 1/sqrt(fan_in))  (torch default, untouched by
    weights_init_normal)
"""
from __future__ import annotations

import math

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _splitmix64(counter: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = counter * _GOLDEN + _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def _stream_key(seed: int, name: str) -> np.uint64:
    h = np.uint64(seed & 0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        for ch in name.encode():
            h = _splitmix64(np.array([h ^ np.uint64(ch)], dtype=np.uint64))[0]
    return h


def uniform(seed: int, name: str, shape, lo: float = 0.0, hi: float = 1.0) -> np.ndarray:
    """U[lo, hi) float32 array, a pure function of (seed, name, shape)."""
    n = int(np.prod(shape)) if len(shape) else 1
    key = _stream_key(seed, name)
    with np.errstate(over="ignore"):
        ctr = np.arange(n, dtype=np.uint64) + key * np.uint64(0x100000001B3)
    bits = _splitmix64(ctr) >> np.uint64(40)  # 24 random bits
    u = bits.astype(np.float64) / float(1 << 24)
    return (lo + (hi - lo) * u).astype(np.float32).reshape(shape)


def normal(seed: int, name: str, shape, mean: float = 0.0, std: float = 1.0) -> np.ndarray:
    """N(mean, std) float32 array via Box-Muller on two independent streams."""
    n = int(np.prod(shape)) if len(shape) else 1
    u1 = uniform(seed, name + "#u1", (n,)).astype(np.float64)
    u2 = uniform(seed, name + "#u2", (n,)).astype(np.float64)
    u1 = np.maximum(u1, 1.0 / (1 << 24))
    z = np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * math.pi * u2)
    return (mean + std * z).astype(np.float32).reshape(shape)


def bernoulli(seed: int, name: str, shape, p: float) -> np.ndarray:
    return (uniform(seed, name, shape) < p).astype(np.float32)


def init_state_dict(shapes: dict, seed: int) -> dict:
    """Deterministic state_dict for a model given {name: shape} in state_dict order.

    Conv weights (4-d) ~ N(0, 0.02); 1-d biases ~ U(+-1/sqrt(fan_in)) where fan_in is
    taken from the preceding weight of the same layer.
    """
    out = {}
    last_fan_in = 1
    for name, shape in shapes.items():
        shape = tuple(shape)
        if len(shape) == 4:
            out[name] = normal(seed, name, shape, 0.0, 0.02)
            last_fan_in = shape[1] * shape[2] * shape[3]
        elif len(shape) == 1:
            b = 1.0 / math.sqrt(last_fan_in)
            out[name] = uniform(seed, name, shape, -b, b)
        else:
            raise ValueError(f"unexpected parameter shape {name}: {shape}")
    return out


def step_model_seeds(seed: int) -> dict:
    """Per-model seeds of the multi-step golden fixture (tests/golden/make_golden.py)."""
    return {tag: seed + len(tag) * 31 + sum(map(ord, tag)) for tag in ("G_A2B", "G_B2A", "D_A", "D_B")}
