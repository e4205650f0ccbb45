"""CPU: pin the refinement oracle (oracle/sgd_ref.py) to the reference.

Golden vectors were produced by importing the reference's pose_refinement /
utils in the build container (tests/golden/make_golden.py):
* project.npz  — project_points_torch (pose_refinement.py:94-179), with and
                 without distortion, and with an axis-angle R;
* bodylen.npz  — utils.get_body_part_lengths (utils.py:1185-1208);
* sgd_*.npz    — Optimized_3d_Pose_Estimation.sgd_optimize (:894-1096):
                 whole-sequence and windowed (batch 8) runs, V=2/8, and an
                 early-stopping run (patience 3, tolerance 0.2).
The oracle must reproduce all of them bit-exactly (same torch ops on CPU).
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import sgd_ref

# examples/body_part_lengths.yaml:my_lengths of the reference (key order kept)
with open(os.path.join(GOLDEN, "body_part_lengths.json")) as _f:
    MY_LENGTHS = json.load(_f)["my_lengths"]

SGD_CASES = ["sgd_V2_T40", "sgd_V2_T40_b8", "sgd_V8_T20", "sgd_V2_T24_stop"]


def sgd_kwargs(d):
    kw = {k: (None if np.isnan(v) else float(v)) for k, v in zip(d["kw_names"], d["kw_vals"])}
    for k in ("patience", "max_iter", "batch_size"):
        if kw.get(k) is not None:
            kw[k] = int(kw[k])
    return kw


def sgd_cams(d):
    return [[d["K"][v], d["R"][v], d["T"][v], d["dist"][v]] for v in range(d["K"].shape[0])]


def test_project_points_matches_reference():
    d = np.load(os.path.join(GOLDEN, "project.npz"))
    pts = torch.tensor(d["points"])
    for v in range(3):
        for ign in (0, 1):
            out = sgd_ref.project_points(pts, d["K"][v], d["R"][v], d["T"][v], d["dist"][v],
                                         ignore_distortions=bool(ign))
            np.testing.assert_array_equal(out.numpy(), d[f"out_c{v}_{ign}"])
    out = sgd_ref.project_points(pts, d["K"][1], torch.tensor(d["rvec"], dtype=torch.float32), d["T"][1],
                                 d["dist"][1])
    np.testing.assert_array_equal(out.numpy(), d["out_axisangle"])


def test_body_part_lengths_match_reference():
    d = np.load(os.path.join(GOLDEN, "bodylen.npz"))
    L = sgd_ref.body_part_lengths(torch.tensor(d["poses"]))
    assert list(L.keys()) == list(d["names"])
    np.testing.assert_array_equal(np.stack([L[n].numpy() for n in d["names"]]), d["lengths"])


@pytest.mark.parametrize("case", SGD_CASES)
def test_sgd_matches_reference(case):
    d = np.load(os.path.join(GOLDEN, case + ".npz"))
    r = sgd_ref.refine(d["gauss"], d["init"], sgd_cams(d), body_lengths=dict(MY_LENGTHS), **sgd_kwargs(d))
    np.testing.assert_array_equal(r.best_trajectory.numpy(), d["best"])
    np.testing.assert_array_equal(r.trajectory.numpy(), d["final"])
    for k, v in r.all_costs_total.items():
        np.testing.assert_array_equal(np.array([float(x) for x in v]), d["hist_" + k])


@pytest.mark.parametrize("case,kw", [("default", {}), ("rolling", dict(use_rolling_average=True)),
                                     ("nomedian", dict(filter_distance_from_median=False)),
                                     ("k7", dict(k=7, k_std=1.5, median_std=3))])
def test_linear_interpolation_matches_reference(case, kw):
    from oracle import interp_ref
    d = np.load(os.path.join(GOLDEN, "interp.npz"))
    np.testing.assert_array_equal(interp_ref.linear_interpolation(d["points"], **kw), d["out_" + case])


C5_CASES = ["sgd_V8_T400", "sgd_V8_T400_b100", "sgd_V8_T400_stop"]


def c5_problem(d):
    """Rebuild a config-5 golden's inputs from its seed and check them against the digest the
    generator recorded (the 2.6 MB inputs are not stored)."""
    from sgd_problem import inputs_digest, sgd_inputs
    cams, gauss, init = sgd_inputs(int(d["V"][0]), int(d["T"][0]), int(d["seeds"][0]))
    assert inputs_digest(cams, gauss, init) == str(d["digest"]), "synthetic problem generator drifted"
    return [[c["K"], c["R"], c["T"], c["dist"]] for c in cams], gauss, init


@pytest.mark.parametrize("case", C5_CASES)
def test_sgd_config5_matches_reference(case):
    """BASELINE config 5 (V=8, T=400): one window, windows of 100, early stop (317 iterations)."""
    d = np.load(os.path.join(GOLDEN, case + ".npz"))
    cams, gauss, init = c5_problem(d)
    r = sgd_ref.refine(gauss, init, cams, body_lengths=dict(MY_LENGTHS), **sgd_kwargs(d))
    np.testing.assert_array_equal(r.best_trajectory.numpy(), d["best"])
    np.testing.assert_array_equal(r.trajectory.numpy(), d["final"])
    for k, v in r.all_costs_total.items():
        np.testing.assert_array_equal(np.array([float(x) for x in v]), d["hist_" + k])
