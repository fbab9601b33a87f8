"""The vectorised torch port (oracle/v9_torch_port.py, the CPU-baseline workload) computes the
reference's values: pinned to the golden sums and to the C oracle's per-product terms."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc
from oracle import v9_torch_port as port
from tests import golden_io as gio

META = gio.meta()


@pytest.mark.parametrize("case", [c for c in META["g2"] if c["fmt"] != "E5M2"][::3], ids=lambda c: c["key"])
def test_port_matches_golden(case):
    g = gio.load("g2_matmul.npz")
    A = torch.from_numpy(g[case["fmt"] + "_A"][:16])
    B = torch.from_numpy(g[case["fmt"] + "_B"][:, :8])
    tab = torch.from_numpy(g[f"{case['fmt']}_table_{case['table']}"])
    C = port.matmul(A, B, case["E"], case["M"], case["bA"], case["bB"], case["bR"], tab, approx=case["approx"],
                    s2n=case["s2n"], qbma=case["qbma"], gclip=case["gclip"]).numpy()
    ref, S = orc.matmul(A.numpy(), B.numpy(), case["E"], case["M"], case["bA"], case["bB"], case["bR"], tab.numpy(),
                        gio.flags_from(case), with_abs=True)
    assert np.all(np.abs(C - ref) <= gio.sum_tolerance(S))
    assert np.all(np.abs(C - g[case["key"] + "_C"][:16, :8]) <= gio.sum_tolerance(S))
