"""Generate the committed golden fixtures (run offline in the dev container; test infrastructure).

For each case the CPU oracle renders the frame; on the small frames it is first cross-checked
BIT FOR BIT against the independent pure-Python restatement (oracle/pyref.py).  Written:

  tests/golden/frames.npz     uint8 RGBA frames, key = case id
  tests/golden/samples.npz    f64 RGBA of a fixed pseudo-random set of pixels per case
                              (key "<case>" -> (n, 6) rows: x, y, r, g, b, a)
  tests/golden/index.json     case parameters, sha256 of every frame, whether pyref agreed

The reference itself ships no golden images and cannot be built here, so these
fixtures pin the oracle to its own cross-checked output ("parity unpinned" against the Rust
binary; see DESIGN.md "Oracle").
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from oracle import pyref as P  # noqa: E402

SCENES = os.path.join(HERE, "scenes")

# (case id, scene name or inline text, time, W, H, max_depth, cross-check with pyref)
CASES = [
    ("globes_64x48_t0", "globes", 0.0, 64, 48, 10, True),
    ("globes_160x120_t0", "globes", 0.0, 160, 120, 10, False),
    ("globes_160x120_t0.25", "globes", 0.25, 160, 120, 10, False),
    ("globes_160x120_t0.5", "globes", 0.5, 160, 120, 10, False),
    ("globes_320x240_d5", "globes", 0.0, 320, 240, 5, False),
    ("spinning_globes_160x120_t0.1", "spinning_globes", 0.1, 160, 120, 10, False),
    ("spinning_globes_48x36_t0.1", "spinning_globes", 0.1, 48, 36, 10, True),
    ("sphere_192x108_d0", "draw(sphere(<0, 0, 0>, 30, red))", 0.0, 192, 108, 0, True),
    ("three_cubes_96x72", "three_cubes", 0.0, 96, 72, 10, True),
    ("spinning_cube_96x72_t0.3", "spinning_cube", 0.3, 96, 72, 10, True),
    ("ground_star_96x72_t0.2", "ground_star", 0.2, 96, 72, 10, True),
    ("spinning_gimbals_96x72_t0.4", "spinning_gimbals", 0.4, 96, 72, 10, False),
    ("spinning_gimbals_32x24_t0.4", "spinning_gimbals", 0.4, 32, 24, 10, True),
    ("fractal_96x72", "fractal", 0.0, 96, 72, 10, False),
    ("fractal_16x12", "fractal", 0.0, 16, 12, 10, True),
]


def scene_text(s):
    path = os.path.join(SCENES, s + ".scene")
    return open(path).read() if os.path.exists(path) else s


def main():
    tex = O.register_texture_file("worldmap.png", os.path.join(SCENES, "worldmap.png"))
    ptex = {"worldmap.png": P.load_texture(tex)}
    frames, samples, index = {}, {}, {}
    rng = np.random.default_rng(20261015)
    for cid, scene, t, W, H, depth, cross in CASES:
        text = scene_text(scene)
        sc = O.OracleScene(text, t, W, H, max_depth=depth)
        f, u = sc.render(f64=True, threads=8)
        agreed = None
        if cross:
            py = P.Scene(text, t, W, H, ptex, max_depth=depth)
            pf = np.array([[[c.r, c.g, c.b, c.a] for c in row] for row in py.render()])
            agreed = bool(np.array_equal(pf, f))
            if not agreed:
                raise SystemExit(f"{cid}: oracle and pyref disagree (max {np.abs(pf - f).max()})")
        n = min(300, W * H)
        idx = rng.choice(W * H, size=n, replace=False)
        ys, xs = np.divmod(idx, W)
        samples[cid] = np.column_stack([xs, ys, f[ys, xs]]).astype(np.float64)
        frames[cid] = u
        index[cid] = {"scene": scene, "time": t, "width": W, "height": H, "max_depth": depth,
                      "sha256_rgba8": hashlib.sha256(u.tobytes()).hexdigest(),
                      "pyref_bit_equal_f64": agreed}
        print(cid, index[cid]["sha256_rgba8"][:16], "pyref:", agreed, flush=True)
    np.savez_compressed(os.path.join(HERE, "frames.npz"), **frames)
    np.savez_compressed(os.path.join(HERE, "samples.npz"), **samples)
    with open(os.path.join(HERE, "index.json"), "w") as fh:
        json.dump(index, fh, indent=1)


if __name__ == "__main__":
    main()
