"""Helpers shared by the tests."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def bits(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def assert_bits_equal(got, want, what="array"):
    """Bit-exact float32 equality; NaNs must sit at the same places (payloads may differ)."""
    got = np.ascontiguousarray(got, dtype=np.float32)
    want = np.ascontiguousarray(want, dtype=np.float32)
    assert got.shape == want.shape, f"{what}: shape {got.shape} != {want.shape}"
    gn, wn = np.isnan(got), np.isnan(want)
    assert (gn == wn).all(), f"{what}: NaN positions differ ({int((gn != wn).sum())} places)"
    ok = bits(got)[~gn] == bits(want)[~wn]
    if not ok.all():
        idx = np.argwhere(~ok.reshape(-1))[:5].ravel()
        g, w = got[~gn].ravel()[idx], want[~wn].ravel()[idx]
        raise AssertionError(f"{what}: {int((~ok).sum())} of {ok.size} values differ in bits, e.g. {g} vs {w}")


def assert_values_equal(got, want, what="array"):
    """Value equality (+0 == -0), NaN-aware -- for scales, whose zero sign never reaches O."""
    got = np.asarray(got, dtype=np.float32)
    want = np.asarray(want, dtype=np.float32)
    assert got.shape == want.shape, f"{what}: shape {got.shape} != {want.shape}"
    gn, wn = np.isnan(got), np.isnan(want)
    assert (gn == wn).all(), f"{what}: NaN positions differ"
    assert (got[~gn] == want[~wn]).all(), f"{what}: values differ"


def load_kat():
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        return json.load(f)


def load_cases():
    with open(os.path.join(GOLDEN, "cases.json")) as f:
        index = json.load(f)
    arrays = np.load(os.path.join(GOLDEN, "cases.npz"))
    return index, arrays
