"""Loss terms of three f16 / f16x3 training steps of the concurrent soft + lung pair on the steps_64
fixture's seeds, written as exact float reprs, for a bit-exactness comparison of two library builds
(run once per build with DUCOSY_HIP_LIB set; later steps depend on every earlier gradient and update):

    python scripts/diag/step_losses.py OUT.json [--mma f16]     then     python scripts/diag/step_losses.py --cmp A.json B.json
"""
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "ducosy-gan_amd")]


def main():
    if sys.argv[1] == "--cmp":
        a, b = (json.load(open(f)) for f in sys.argv[2:4])
        bad = [k for k in a if a[k] != b[k]]
        for k in bad:
            print("DIFF", k, a[k], b[k])
        print("identical" if not bad else f"{len(bad)} of {len(a)} differ", len(a))
        sys.exit(1 if bad else 0)
    import numpy as np
    from conftest import GOLDEN
    from oracle import prng
    from test_gpu_concurrent import _batch
    from test_gpu_train import _system
    from modules.hip import ops
    from modules.trainer import ConcurrentCycleGANs
    mma = sys.argv[sys.argv.index("--mma") + 1] if "--mma" in sys.argv else "f16"
    z = np.load(os.path.join(GOLDEN, "steps_64.npz"))
    n, hw, nb, cin, steps, seed = [int(v) for v in z["meta"]]
    lung_seed = 813
    ops.set_mma(mma)
    run = ConcurrentCycleGANs([_system(cin, nb, prng.step_model_seeds(seed)),
                               _system(2, nb, prng.step_model_seeds(lung_seed))], "cuda")
    out = {}
    for i in range(3):
        res = run.train_step([_batch(seed, i, n, hw, cin), _batch(lung_seed, i, n, hw, 2)])
        for m, o in zip(("soft", "lung"), res):
            for k, v in o.items():
                out[f"{i}/{m}/{k}"] = repr(float(v))
    json.dump(out, open(sys.argv[1], "w"), indent=0)
    print(len(out), "terms")


if __name__ == "__main__":
    main()
