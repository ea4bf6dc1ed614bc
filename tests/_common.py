"""Helpers shared by the CPU and GPU tests: scene setup and the parity comparison."""
from __future__ import annotations

import functools

import numpy as np

import dxrpathtracer_amd as D
from oracle import pyoracle as O

# Parity gate (BASELINE.json north_star): per-pixel RGB within 1e-4 relative at matched CMJ indices.
# The relative error's denominator is floored at ATOL / RTOL = 1e-4 (radiance is in 2^-10-scaled units,
# sky texels ~1..5), so the gate is relative for every pixel brighter than 1e-4 and 1e-8 absolute below.
RTOL = 1e-4
ATOL = 1e-8
# max relative error seen per parity check in this session (reported by conftest's terminal summary)
PARITY_LOG: list = []


@functools.lru_cache(maxsize=None)
def scene_bundle(name: str, detail: int = 0):
    """(Scene, Sky) for a scene id, cached per test session."""
    sc = D.Scene(name, detail=detail)
    sky = D.make_sky(sc.settings())
    return sc, sky


@functools.lru_cache(maxsize=None)
def oracle_scene(name: str, detail: int = 0):
    sc, sky = scene_bundle(name, detail)
    return O.OracleScene(sc, sky)


def rel_err(gpu: np.ndarray, ref: np.ndarray) -> np.ndarray:
    return np.abs(gpu - ref) / np.maximum(np.abs(ref), ATOL / RTOL)


def assert_parity(gpu: np.ndarray, ref: np.ndarray, what: str):
    assert gpu.shape == ref.shape, (gpu.shape, ref.shape)
    assert np.isfinite(gpu).all(), f"{what}: non-finite GPU pixels"
    e = rel_err(gpu[..., :3], ref[..., :3])
    PARITY_LOG.append((what, float(e.max()) if e.size else 0.0, int(e.shape[0] * e.shape[1])))
    bad = e > RTOL
    if bad.any():
        idx = np.argwhere(bad)[:5]
        detail = ", ".join(f"{tuple(i)} gpu={gpu[tuple(i[:2])][:3]} ref={ref[tuple(i[:2])][:3]}" for i in idx)
        raise AssertionError(f"{what}: {int(bad.any(axis=-1).sum())} of {bad.shape[0] * bad.shape[1]} pixels "
                             f"exceed rel {RTOL} (max {e.max():.3e}); first: {detail}")
    assert np.all(gpu[..., 3] == 1.0), f"{what}: alpha must be 1 (RayTrace.hlsl:148)"
