"""Probe: torch (its bundled HIP runtime) and libptx.so (/opt/rocm's) in one process.
usage: python tools/torch_interop_check.py torch-first|ptx-first"""
import sys
import time

order = sys.argv[1]


def use_torch():
    import torch
    ok = torch.cuda.is_available()
    x = torch.arange(8, device="cuda", dtype=torch.float32) * 2 if ok else None
    return ok, (x.sum().item() if ok else None), torch.cuda.device_count()


def use_ptx():
    sys.path.insert(0, ".")
    sys.path.insert(0, "tests")
    from helpers import uniform_for
    from pathtracerdemo_amd.renderer import Renderer
    from pathtracerdemo_amd.scene.world import compile_scene
    cs = compile_scene("dummy_scene_1")
    r = Renderer(32, 32, device=0)
    r.Initialize(cs)
    r.Update()
    r.Render()
    img = r.read_image()
    return float(img.mean())


t = time.time()
if order == "torch-first":
    print("torch", use_torch(), flush=True)
    print("ptx", use_ptx(), flush=True)
    print("torch again", use_torch(), flush=True)
else:
    print("ptx", use_ptx(), flush=True)
    print("torch", use_torch(), flush=True)
print("ok %.1fs" % (time.time() - t))
