"""Offline register / scratch report of the scene-specialised kernels (csrc/spec.hip): dumps the
program rt_scene_spec_program returns for a scene, splits it into one file per kernel (as spec.hip
compiles them), compiles each with hipcc for gfx950 with the hipRTC options and prints the
compiler's resource-usage remarks (VGPRs, spills, scratch bytes per lane, occupancy, LDS).

  RT_LIB_PATH=tinyraytracerinrust_amd/build/librt_mi355x_kl4.so python3 tools/spec_resources.py globes 3840 2160 /tmp/spec_res rows_00
  FAMILY=120 python3 tools/spec_resources.py spinning_globes 1920 1080   (the animation's family program)
"""
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
os.environ.setdefault("RT_NO_TORCH_PRELOAD", "1")


def main():
    import tinyraytracerinrust_amd as T
    from tests.conftest import SCENES, scene_text
    name = sys.argv[1] if len(sys.argv) > 1 else "globes"
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 3840
    H = int(sys.argv[3]) if len(sys.argv) > 3 else 2160
    out = sys.argv[4] if len(sys.argv) > 4 else "/tmp/spec_res"
    only = sys.argv[5] if len(sys.argv) > 5 else None          # regex on the kernel names
    os.makedirs(out, exist_ok=True)
    fam = int(os.environ.get("FAMILY", "0"))          # > 0: the program of a FAMILY-frame animation's family
    if fam:
        frames = [T.Scene.compile(scene_text(name), f / fam, W, H, asset_dir=SCENES) for f in range(fam)]
        T.Scene.register_family(frames)
        text = frames[fam // 2].spec_program()
    else:
        text = T.Scene.compile(scene_text(name), 0.0, W, H, asset_dir=SCENES).spec_program()
    cut = text.index('extern "C" __global__')
    prelude, kernels = text[:cut], text[cut:]
    csrc = os.path.join(ROOT, "tinyraytracerinrust_amd", "csrc")
    for k in re.split(r'(?=extern "C" __global__)', kernels):
        if not k.strip():
            continue
        kname = re.search(r"void (rt_spec_\w+)\(", k).group(1)
        if only and not re.search(only, kname):
            continue
        src = os.path.join(out, kname + ".hip")
        with open(src, "w") as f:
            f.write(prelude + k)
        cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
               "-mllvm", "-disable-machine-licm", "--cuda-device-only", "-c", "-o", os.devnull, src,
               "-Rpass-analysis=kernel-resource-usage", "-I", csrc]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            print(r.stderr[-3000:])
            raise SystemExit(f"{kname}: compile failed")
        rem = dict(re.findall(r"remark:\s+(.+?):\s*(\S+)\s*\[-Rpass", r.stderr))
        keys = ["VGPRs", "VGPRs Spill", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "LDS Size [bytes/block]"]
        print(kname, " ".join(f"{k}={rem.get(k, '?')}" for k in keys))


if __name__ == "__main__":
    main()
