"""Diagnostic: render chosen points (get_pixel at fractional positions) through the library named by
$RT_LIB_PATH and compare them with the oracle: one line per point (RGBA8 and f64).
usage: RT_LIB_PATH=... python3 tools/points_check.py SCENE_FILE W H DEPTH x,y [x,y ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import tinyraytracerinrust_amd as T
    from oracle import oracle as O
    from tests.conftest import SCENES
    O.register_texture_file("worldmap.png", os.path.join(SCENES, "worldmap.png"))
    text = open(sys.argv[1]).read()
    W, H, depth = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    pts = [tuple(float(v) for v in a.split(",")) for a in sys.argv[5:]]
    osc = O.OracleScene(text, 0.0, W, H, max_depth=depth)
    r = T.Renderer(0)
    r.upload(T.Scene.compile(text, 0.0, W, H, asset_dir=SCENES))
    g = r.render_points(np.array(pts, dtype=np.float64), max_depth=depth)
    lib = os.path.basename(os.environ.get("RT_LIB_PATH", "librt_mi355x.so"))
    for (x, y), gc in zip(pts, g):
        rc = osc.get_pixel(x, y)
        g8 = [min(255, max(0, int(v * 255.0))) for v in gc[:3]]
        r8 = [min(255, max(0, int(v * 255.0))) for v in rc[:3]]
        print(f"{lib} ({x!r}, {y!r}) gpu {g8} oracle {r8} {'OK' if g8 == r8 else 'DIFF'} max|d| {np.max(np.abs(gc - rc)):.3e}")


if __name__ == "__main__":
    main()
