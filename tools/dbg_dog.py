import sys, numpy as np, torch
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
from test_gpu_configs import bead_stack_torch
from spim_registration_amd import dog
from oracle import dog_ref
for n in (96, 256, 512, 768):
    img = bead_stack_torch((n, n, n), 20140614)
    pts, d = dog.compute(img, sigma=1.8, threshold=0.008, return_dog=True)
    line = f"n={n} gpu peaks {len(pts)} min {img.min():.4f} max {img.max():.4f} dog range {d.min():.4f} {d.max():.4f}"
    if n == 96:
        pk, dref = dog_ref.process_dog(img, 1.8, 0.008)
        line += f" oracle peaks {len(pk)} dog equal {np.array_equal(d, dref)}"
    print(line, flush=True)
