"""Generate the light-path-variant fixtures under tests/golden/bdpt/*.npz.

The variant (khp_bdpt_params, ABI 7) restates KIRK's GLSL
lbb_construction.compute / pt_shade.compute, which KIRK never runs (its GPU
path tracer is dead code) and which ships no outputs, so these are
oracle outputs that freeze the restatement: the flattened scene as arrays, the
render and variant parameters, the frame and the light subpaths of one sample.

    python tests/golden/bdpt/make_golden_bdpt.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(HERE)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import oracle_ffi  # noqa: E402
from ba_pathtracing_fur_amd import scenes as S  # noqa: E402

CASES = {
    # name: (scene factory kwargs, width, height, spp, depth, (light_paths, vertices))
    "bdpt_config1_cornell": (("config1", {}), 32, 24, 3, 5, (64, 4)),
    "bdpt_config2_hairball": (("config2", dict(n_strands=300)), 32, 24, 2, 5, (32, 3)),
    "bdpt_zoo_all_lights": (("zoo", dict(n_strands=200)), 40, 30, 2, 6, (16, 5)),
}
SEED = 0x4B49524B


def make(name):
    (factory, kw), w, h, spp, depth, (ns, nv) = CASES[name]
    sd = S.build_config(factory, width=w, height=h, **kw)
    o = oracle_ffi.Oracle(sd)
    o.set_bdpt(light_paths=ns, vertices=nv)
    img = o.render(w, h, spp, depth, seed=SEED, threads=8)
    lp = o.light_paths(1, seed=SEED)
    out = dict(sd.to_arrays())
    out.update(params=np.uint32([w, h, spp, depth, SEED]), bdpt=np.uint32([ns, nv]), image=img, light_paths=lp)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    return img


if __name__ == "__main__":
    for name in CASES:
        img = make(name)
        print(f"{name}: {img.shape} finite={np.isfinite(img).all(-1).mean():.3f} mean={np.nanmean(img):.4f}")
