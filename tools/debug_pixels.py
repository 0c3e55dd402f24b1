"""Diagnostic: find the pixels where the GPU frame differs from the oracle and dump both ray trees
(rt_record_rays vs the oracle's recorder) to JSON for offline comparison (pyref can re-trace the
same pixel on the CPU).  usage: python tools/debug_pixels.py SCENE TIME W H DEPTH OUT.json"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SCENES = os.path.join(ROOT, "tests", "golden", "scenes")


def recs(arr):
    return [{k: (arr[k][i].tolist() if hasattr(arr[k][i], "tolist") else arr[k][i]) for k in arr.dtype.names}
            for i in range(len(arr))]


def main():
    import torch
    import tinyraytracerinrust_amd as T
    from oracle import oracle as O
    name, t, W, H, depth, out = sys.argv[1], float(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), sys.argv[6]
    text = open(os.path.join(SCENES, name + ".scene")).read()
    O.register_texture_file("worldmap.png", os.path.join(SCENES, "worldmap.png"))
    rt = T.RayTracer(W, H)
    rt.max_depth = depth
    rt.load_scene(text, t, asset_dir=SCENES)
    g = rt.renderer.render_rows(0, H)
    torch.cuda.synchronize()
    g = g.cpu().numpy()
    gf = rt.renderer.render_rows_host(0, H, f64=True)
    sc = O.OracleScene(text, t, W, H, max_depth=depth)
    rf, ru = sc.render(0, H, f64=True)
    bad = np.argwhere((g != ru).any(-1))
    print(f"{len(bad)} pixels differ", flush=True)
    res = []
    for y, x in bad[:12]:
        grec, gcol = rt.renderer.record_rays(float(x), float(y), depth)
        raw, ocol = sc.record_rays(float(x), float(y))
        orec = np.frombuffer(raw.tobytes(), T.RAY_RECORD_DTYPE)
        res.append({"x": int(x), "y": int(y), "gpu_u8": g[y, x].tolist(), "oracle_u8": ru[y, x].tolist(),
                    "gpu_f64": gf[y, x].tolist(), "oracle_f64": rf[y, x].tolist(),
                    "gpu_points_f64": rt.renderer.render_points(np.array([[x, y]], np.float64))[0].tolist(),
                    "gpu_rays": recs(grec), "oracle_rays": recs(orec),
                    "gpu_color": gcol.tolist(), "oracle_color": ocol.tolist()})
        print(json.dumps(res[-1])[:3000], flush=True)
    json.dump({"scene": name, "time": t, "W": W, "H": H, "depth": depth, "n_bad": int(len(bad)), "pixels": res},
              open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
