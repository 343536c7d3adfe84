"""Synthetic descriptor sets for the matching tests (Features<T>::findCorrespondences,
features.h:224-253): FPFH-like rows (three 11-bin blocks, each summing to 100, as
FPFHEstimation::computeFeature normalises them) and SHOT-like rows (352 non-negative values,
unit L2 norm, as SHOTEstimation normalises them), with a target that is a perturbed permutation
of the source plus distractors -- so most rows have a clear mutual nearest neighbour and some
rows are ambiguous."""
import numpy as np


def fpfh_like(rng, n):
    x = rng.gamma(0.6, 1.0, size=(n, 33)).astype(np.float64)
    for b in range(3):
        blk = x[:, 11 * b:11 * b + 11]
        x[:, 11 * b:11 * b + 11] = blk * (100.0 / blk.sum(1, keepdims=True))
    return x.astype(np.float32)


def shot_like(rng, n, d=352):
    x = rng.gamma(0.3, 1.0, size=(n, d)) * (rng.random((n, d)) < 0.4)
    x[:, 0] += 1e-3
    return (x / np.linalg.norm(x, axis=1, keepdims=True)).astype(np.float32)


def pair(kind, ns, nt, seed, noise=0.02):
    rng = np.random.default_rng(seed)
    make = fpfh_like if kind == "fpfh" else shot_like
    src = make(rng, ns)
    m = min(ns, nt) * 3 // 4
    perm = rng.permutation(ns)[:m]
    scale = 100.0 if kind == "fpfh" else 1.0 / 16
    tgt = np.concatenate([src[perm] + (rng.normal(0, noise * scale, (m, src.shape[1]))).astype(np.float32),
                          make(rng, nt - m)])
    order = rng.permutation(nt)
    return src, np.ascontiguousarray(tgt[order]).astype(np.float32)
