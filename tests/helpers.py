"""Shared test helpers: gradient fingerprints and tolerance checks.

A fingerprint of a tensor is (sum, L2 norm, 256 values at seeded indices and
4 projections on seeded uniform[-1,1) vectors), all accumulated in float64.
The golden fixtures store fingerprints of the 34 parameter gradients so they
stay small while still pinning every element statistically.
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import attention as _dropin  # noqa: E402  (root shim that registers the package)

detinit = _dropin._pkg.detinit

NSAMP = 256
NPROJ = 4


def _seed_for(name: str) -> int:
    h = 1469598103934665603
    for ch in name.encode():
        h = ((h ^ ch) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h >> 1


def fingerprint(name: str, arr) -> dict:
    a = np.asarray(arr, dtype=np.float64).reshape(-1)
    n = a.size
    seed = _seed_for(name)
    idx = (detinit.splitmix64(seed, NSAMP) % np.uint64(n)).astype(np.int64)
    proj = np.stack([detinit.uniform_pm(seed + 17 * (k + 1), n, 1.0).astype(np.float64)
                     for k in range(NPROJ)])
    return {
        "sum": np.array(a.sum()),
        "norm": np.array(np.sqrt((a * a).sum())),
        "samp": a[idx],
        "proj": proj @ a,
    }


def fp_keys(prefix: str, name: str):
    return {k: f"{prefix}{k}__{name}" for k in ("sum", "norm", "samp", "proj")}


def store_fp(out: dict, prefix: str, name: str, arr) -> None:
    fp = fingerprint(name, arr)
    for k, key in fp_keys(prefix, name).items():
        out[key] = fp[k]


def check_fp(golden, prefix: str, name: str, arr, rtol: float) -> float:
    """Return the worst relative error of arr's fingerprint vs the stored one.

    Errors are relative to the tensor's own scale (norm of the reference
    gradient, scaled to the statistic), so near-zero sums do not blow up.
    """
    fp = fingerprint(name, arr)
    keys = fp_keys(prefix, name)
    ref_norm = float(golden[keys["norm"]])
    n = np.asarray(arr).size
    scale = max(ref_norm, 1e-30)
    worst = 0.0
    # sums/projections of n terms scale like norm*sqrt(n); samples like norm/sqrt(n)
    worst = max(worst, abs(float(fp["norm"]) - ref_norm) / scale)
    worst = max(worst, abs(float(fp["sum"]) - float(golden[keys["sum"]])) / (scale * np.sqrt(n)))
    worst = max(worst, float(np.max(np.abs(fp["proj"] - golden[keys["proj"]]))) / (scale * np.sqrt(n)))
    smax = max(float(np.max(np.abs(golden[keys["samp"]]))), 1e-30)
    worst = max(worst, float(np.max(np.abs(fp["samp"] - golden[keys["samp"]]))) / smax)
    return worst


def rel_err(x, ref) -> float:
    """Norm-relative error ||x-ref|| / ||ref||."""
    x = np.asarray(x, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    d = np.sqrt(((x - ref) ** 2).sum())
    n = np.sqrt((ref ** 2).sum())
    return float(d / max(n, 1e-30))


def assert_close(x, ref, rtol: float, what: str = "") -> None:
    """Norm-relative error <= rtol AND elementwise |x-ref| <= rtol*max|ref| (+rtol*|ref|)."""
    x = np.asarray(x, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    assert x.shape == ref.shape, f"{what}: shape {x.shape} vs {ref.shape}"
    assert np.all(np.isfinite(x)), f"{what}: non-finite values"
    e = rel_err(x, ref)
    assert e <= rtol, f"{what}: norm-relative error {e:.3e} > {rtol:.1e}"
    atol = rtol * max(float(np.abs(ref).max()), 1e-30)
    bad = np.abs(x - ref) > atol + rtol * np.abs(ref)
    assert not bad.any(), (f"{what}: {int(bad.sum())} elements beyond tolerance; "
                           f"max abs diff {float(np.abs(x - ref).max()):.3e}, atol {atol:.3e}")
