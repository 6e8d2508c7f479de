"""bench.py refuses a step that produced non-finite numbers.

After the timed loop, outside the timing, bench.py reduces the last step's loss terms and every
optimizer's flat parameter buffer to one device-side isfinite verdict, writes it to the JSON line
as "finite", and exits 3 when it is false.  Round 5 showed why: a kernel whose epilogue corrupted
the data gradient's halo produced NaN from the second step on, and NaN operands draw less power, so
the clock rose and the bench read 12 % faster.  Here the bench runs a small full step (64x64, bs 2,
one residual block) once as is and once with a NaN injected into the synthetic inputs."""
import json
import os
import subprocess
import sys

import pytest
import torch

from conftest import ROOT

SMALL = ["--img", "64", "--batch", "2", "--blocks", "1", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]


def _bench(*extra):
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *SMALL, *extra], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=240)


def _record(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out
    return json.loads(lines[-1])


def test_all_finite_helper_cpu():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.all_finite([torch.zeros(3), torch.ones(2, 2), torch.empty(0)])
    assert not bench.all_finite([torch.zeros(3), torch.tensor([1.0, float("nan")])])
    assert not bench.all_finite([torch.tensor(float("inf"))])


@pytest.mark.gpu
def test_bench_reports_finite_step():
    r = _bench()
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _record(r.stdout)
    assert rec["finite"] is True and rec["value"] > 0


@pytest.mark.gpu
def test_bench_exits_nonzero_on_nan_step():
    r = _bench("--inject-nan")
    assert r.returncode == 3, (r.returncode, r.stderr[-3000:])
    rec = _record(r.stdout)
    assert rec["finite"] is False
    assert "non-finite" in r.stderr
