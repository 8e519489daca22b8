"""Shared pytest setup: repo on sys.path, the `gpu` marker, golden fixtures.

CPU tests (-m "not gpu") cover the oracle against the reference's golden
vectors, the host logic, and the C-ABI library's load/exports.  GPU tests
(-m gpu) are the parity tests proper and call the HIP path through the C ABI.
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


def _load(name):
    with open(os.path.join(GOLDEN, name)) as fh:
        return json.load(fh)


@pytest.fixture(scope="session")
def scenario():
    return _load("reference_scenario.json")


@pytest.fixture(scope="session")
def units():
    return _load("reference_units.json")


@pytest.fixture(scope="session")
def candidates():
    return _load("reference_candidates.json")


@pytest.fixture(scope="session")
def oracle():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    from oracle import oracle as O
    return O


@pytest.fixture(scope="session")
def engine():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from diplomjourney_amd.expansion import Expansion
    return Expansion("cuda:0")


def call_problem(rec):
    """mpc_problem_t of one recorded predictive_control call."""
    from diplomjourney_amd.abi import make_problem
    pre, t = rec["pre"], rec["post"]["t"]
    return make_problem(rec["x"], rec["y"], rec["phi"], pre["x_t"], pre["y_t"], pre["x_0"],
                        pre["y_0"], 0.5, t, t + 0.05)


def call_controls(rec, n_steps=3):
    """Candidate SoA of one recorded call, with the slow-down override (:312-316)."""
    import numpy as np
    V, B = list(rec["V"]), list(rec["B"])
    if rec["pre"]["steps_for_slowing"] > 0:
        V = [min(V) if min(V) > 0.4 else 0.4] * len(V)
    vv = np.repeat(np.array(V, dtype=np.float64), len(B))
    bb = np.tile(np.array(B, dtype=np.float64), len(V))
    return np.tile(vv, (n_steps, 1)), np.tile(bb, (n_steps, 1))
