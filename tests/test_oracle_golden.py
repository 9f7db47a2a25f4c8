"""The oracle (CPU restatement) checked against the committed golden fixtures.

gp_cases.npz / c1.npz come from numpy/scipy fp64 AND scikit-learn (asserted to
agree in tests/golden/make_golden.py); contours.json are hand-derived from
OpenCV 4.5.x's RETR_EXTERNAL/CHAIN_APPROX_NONE border follower."""
import numpy as np
import pytest

from oracle import oracle as O


def _hyper(c):
    ell, sf, sn2, m0 = c["hyper"]
    return float(ell), float(sf) ** 2, float(sn2), float(m0)


@pytest.mark.parametrize("name", ["lpsc", "syn256", "syn1024"])
def test_gp_matches_golden(gp_cases, name):
    c = gp_cases[name]
    ell, sf2, sn2, m0 = _hyper(c)
    Lcm, alpha = O.fit(c["x"], c["y"], c["obs"], ell, sf2, sn2, m0)
    mu, var = O.predict(Lcm, alpha, c["x"], c["y"], c["qx"], c["qy"], ell, sf2, m0)
    assert np.abs(mu - c["mu"]).max() <= 1e-9 * max(1.0, np.abs(c["mu"]).max())
    assert np.abs(var - c["var"]).max() <= 1e-9


def test_c1_matches_golden(c1_case):
    c = c1_case
    ell, sf2, sn2, m0 = _hyper(c)
    Lcm, alpha = O.fit(c["x"], c["y"], c["obs"], ell, sf2, sn2, m0)
    mu, var = O.predict(Lcm, alpha, c["x"], c["y"], c["qx"], c["qy"], ell, sf2, m0)
    assert np.abs(mu - c["mu"]).max() <= 1e-9 * np.abs(c["mu"]).max()
    assert np.abs(var - c["var"]).max() <= 1e-9


@pytest.mark.parametrize("name", ["lpsc", "syn256", "syn1024"])
def test_compute_sets_bit_exact(gp_cases, name):
    c = gp_cases[name]
    lo, hi, s = O.compute_sets(c["mu"], c["sd"], float(c["beta"]), float(c["f_min"]))
    assert np.array_equal(lo, c["lo"]) and np.array_equal(hi, c["hi"]) and np.array_equal(s, c["safe"])


def test_contours_known_answers(contour_cases):
    for case in contour_cases:
        img = np.array(case["mask"], np.uint8)
        got = [c.tolist() for c in O.find_contours_external(img)]
        assert got == case["contours"], case["name"]


def test_rbf_fill_formulations_agree():
    rng = np.random.default_rng(0)
    x = rng.uniform(0, 3, 64).astype(np.float32)
    y = rng.uniform(0, 3, 64).astype(np.float32)
    K32 = O.rbf_fill_f32(x, y)
    K64 = O.rbf_fill_f32in(x, y)
    assert np.abs(K32 - K64).max() < 2e-5
    assert np.allclose(np.diag(K64), 1.1)


def test_cholesky_backward_error():
    rng = np.random.default_rng(1)
    x = rng.uniform(0, 4, 300); y = rng.uniform(0, 4, 300)
    K = O.rbf_fill(x, y)
    L = O.lower_from_colmajor(O.cholesky(K))
    assert np.abs(L @ L.T - K).max() < 1e-12
    with pytest.raises(np.linalg.LinAlgError):
        O.cholesky(-np.eye(3))


def test_argmax_semantics():
    s = np.array([1.0, 3.0, np.nan, 3.0, 2.0])
    assert O.argmax(s) == (1, 3.0)                      # lowest index on ties, NaN never wins
    assert O.argmax(s, np.array([1, 0, 1, 1, 1], np.uint8))[0] == 3
    assert O.argmax(s, np.zeros(5, np.uint8))[0] == -1


def test_subgoal_on_c1(c1_case):
    c = c1_case
    w, h = int(c["width"]), int(c["height"])
    F = O.find_safety_contour_indices(c["qx"], c["qy"], c["safe"], w, h)
    assert F.size > 0 and np.all(c["safe"][F] == 1)
    idx = O.next_subgoal(c["qx"], c["qy"], c["lo"], c["hi"], c["safe"], w, h, 0.0, 0.0)
    assert idx in set(F.tolist())
    # f_min from config/safe_bayesian_optimization.yaml:6 (500) makes every cell unsafe -> -1
    lo, hi, s = O.compute_sets(c["mu"], c["sd"], 2.0, 500.0)
    assert s.sum() == 0
    assert O.next_subgoal(c["qx"], c["qy"], lo, hi, s, w, h) == -1
