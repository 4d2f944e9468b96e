"""Generates the committed golden vectors under tests/golden/ from the oracle.

    python tests/golden/make_golden.py

PARITY UNPINNED: the Java reference cannot run in this container (no JVM, no
ImgLib2 jars) and ships no fixtures, so these vectors come
from the CPU restatement in ``oracle/`` (deterministic seeds; see each case).
They freeze the oracle's behaviour: the CPU suite checks the oracle still
reproduces them, the GPU suite checks the HIP path against them.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import dog_ref, mvdecon_ref as ref  # noqa: E402
from spim_registration_amd import synthetic  # noqa: E402

RL_CASES = [
    # name, shape (z,y,x), views, ksize (x,y,z), psftype, iters, lambda, weights, partial, T
    ("rl_independent_l0", (16, 18, 20), 2, (5, 7, 9), ref.PSFTYPE.INDEPENDENT, 4, 0.0, "ones", False, 8),
    ("rl_opt1_tikhonov_partial", (16, 18, 20), 3, (5, 7, 9), ref.PSFTYPE.OPTIMIZATION_I, 4, 0.006, "blend", True, 8),
    ("rl_opt2_T4", (14, 16, 18), 3, (7, 5, 9), ref.PSFTYPE.OPTIMIZATION_II, 3, 0.006, "blend", False, 4),
    ("rl_bayes_T1", (14, 16, 18), 3, (5, 5, 7), ref.PSFTYPE.EFFICIENT_BAYESIAN, 3, 0.006, "blend", True, 1),
]


def make_rl():
    for i, (name, shape, V, ks, pt, iters, lam, wt, partial, T) in enumerate(RL_CASES):
        imgs, ws, psfs, _ = synthetic.make_views(shape, V, config_id=100 + i, ksize=ks, weights=wt,
                                                 partial=partial, bead_density=1.0 / 6 ** 3)
        k1, k2 = ref.prepare_kernels(psfs, pt, T)
        res = ref.mv_deconvolution(imgs, ws, psfs, pt, iters, lam, ij_threads=T)
        np.savez_compressed(os.path.join(HERE, name + ".npz"),
                            imgs=np.stack(imgs), weights=np.stack(ws), psfs=np.stack(psfs),
                            k1=np.stack(k1), k2=np.stack(k2), psi=res.psi,
                            stats=np.array(res.stats, np.float64), avg=np.float64(res.avg),
                            psftype=np.int32(pt), iters=np.int32(iters), lam=np.float64(lam),
                            ij_threads=np.int32(T))


def make_conv():
    rng = np.random.default_rng(5)
    a = rng.random((19, 21, 23)).astype(np.float32)
    k = synthetic.psf(2, 5, (7, 9, 5))
    blk = rng.random((20, 22, 24)).astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "conv.npz"), a=a, k=k,
                        mirror=ref.convolve(a, k, "mirror"), one=ref.convolve(a, k, "one"),
                        block=blk, circular=ref.circular_convolve_block(blk, k))


def make_dog():
    rng = synthetic.rng_for(55)
    shape = (28, 30, 32)
    t = synthetic.truth_volume(shape, rng, bead_density=1.0 / 9 ** 3)
    k = synthetic.psf(0, 1, (7, 7, 11), sigma=(1.0, 1.0, 1.6))
    img = ref.convolve(t.astype(np.float32), k, "mirror")
    img = (rng.poisson(np.maximum(img * 2000 + 50, 0))).astype(np.float32)
    peaks, dog = dog_ref.process_dog(img, 1.8, 0.008)
    np.savez_compressed(os.path.join(HERE, "dog.npz"), img=img, dog=dog,
                        peaks=np.array([p[:3] for p in peaks], np.int32).reshape(-1, 3),
                        intensity=np.array([p[3] for p in peaks], np.float32))


if __name__ == "__main__":
    make_rl()
    make_conv()
    make_dog()
    print("golden vectors written to", HERE)
