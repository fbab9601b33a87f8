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


def v5_case(c):
    """(A, B, table, flags) of a G7 (approx_matmul_whole_v5) case."""
    g = load("g7_v5.npz")
    bk = c["key"].rsplit("_", 2)[0]
    M = c["M"]
    tab = np.zeros((2 ** M, 2 ** M), np.int32) if c["table"] == "zero" else g[f"{c['fmt']}_table_{c['table']}"]
    flags = 32 | (64 if c["ofuf"] else 0) | (128 if c["of_opt"] else 0) | (256 if c["uf_opt"] else 0)
    return g[bk + "_A"], g[bk + "_B"], np.ascontiguousarray(tab, np.int32), flags
