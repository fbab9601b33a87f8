"""Shared helpers for reading tests/golden fixtures (data only, no reference code)."""
import json
import os

import numpy as np

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(HERE, name), allow_pickle=False)


def meta():
    with open(os.path.join(HERE, "meta.json")) as f:
        return json.load(f)


def flags_from(c, tb=False):
    return (1 if c["approx"] else 0) | (2 if c["s2n"] else 0) | (4 if c["qbma"] else 0) | \
        (8 if c.get("gclip", False) else 0) | (16 if tb else 0)


def sum_tolerance(abs_sum):
    """|c - c_hat| <= 1e-5 * sum_k |v_k| + tiny (summation order differs)."""
    return 1e-5 * abs_sum + 1e-30
