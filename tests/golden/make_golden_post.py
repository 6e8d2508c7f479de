"""Golden outputs of the reference's modules/postprocess.py (generate.py's volume
post-processing) for tests/test_cpu_postprocess.py.

Run ONLY in the build container, where /root/reference exists:

    python tests/golden/make_golden_post.py      # writes tests/golden/postprocess.npz

The reference module needs only numpy and scipy; it is imported from its file and called on a
small synthetic CT-like volume.  Only inputs and outputs are written.
"""
import importlib.util
import os

import numpy as np

REF = os.environ.get("DUCOSY_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def volume(seed, shape=(7, 20, 18)):
    rng = np.random.default_rng(seed)
    v = rng.normal(40, 300, shape)
    v[:, 4:9, 5:11] += 900        # a bone-like block above the 750 HU threshold
    v[2] += 400                    # a bright slice (z steps)
    return v.astype(np.float32)


def main():
    spec = importlib.util.spec_from_file_location("ref_postprocess", os.path.join(REF, "modules", "postprocess.py"))
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)
    v = volume(1)
    out = {"volume": v}
    cases = {
        "gaussian": dict(method="gaussian"),
        "gaussian_s2": dict(method="gaussian", sigma=2.0, enhance_sharpness=False),
        "gaussian3d": dict(method="gaussian3d"),
        "gaussian3d_synth": dict(method="gaussian3d", sigma_z=0.7, sigma_xy=0.05, enhance_sharpness=True,
                                 sharpen_amount=1.7, sharpen_radius=1.2),  # generate.py:251-253
        "adaptive": dict(method="adaptive"),
        "median": dict(method="median", enhance_sharpness=False),
        "median5": dict(method="median", kernel_size=5),
        "interpolation": dict(method="interpolation"),
        "kalman": dict(method="kalman"),
        "kalman_q": dict(method="kalman", process_variance=1e-3, measurement_variance=1e-1, enhance_sharpness=False),
        "thr500": dict(method="gaussian3d", hu_threshold=500),
    }
    for name, kw in cases.items():
        out[f"post:{name}"] = ref.postprocess_ct_volume(v.copy(), **kw)
    v2 = volume(2)
    out["volume2"] = v2
    out["unsharp"] = ref.unsharp_mask(v2, v, amount=0.8, radius=1.5)
    out["kalman1d"] = ref.kalman_filter_1d(v[:, 3, 3].astype(np.float64), 1e-5, 1e-2)
    diff = np.abs(volume(3)).astype(np.float32) % 20
    out["diff"] = diff
    out["diffmap"] = ref.apply_diffmap(v.copy(), diff.copy(), threshold=8)
    # the synthesis stage as generate.py:246-254 runs it
    z = ref.gaussian_filter1d(v, sigma=0.8, axis=0)
    out["synth"] = ref.postprocess_ct_volume(z, method="gaussian3d", sigma_z=0.7, sigma_xy=0.05,
                                             enhance_sharpness=True, sharpen_amount=1.7, sharpen_radius=1.2)
    np.savez_compressed(os.path.join(OUT, "postprocess.npz"), **out)
    print("wrote", os.path.join(OUT, "postprocess.npz"))


if __name__ == "__main__":
    main()
