"""The fit's run-time accuracy guard of its f64 inverse (SBO_OPT_INV_CHECK,
round 5) and the posterior on ill-conditioned K where the int8-sliced inverse
runs (N > 4096: csrc/ozgemm.hip at the recursion's splits >= 4096; N = 16384
slices both top levels).

The sliced GEMM's error is relative to row and column maxima, so its effect
grows with cond(K), which the mapper's configuration sets
(config/lpsc.yaml:35-37: noise_level, length_scale).  The precision probe
cannot see it (its fast and precise sweeps read the same inverse); the guard
measures it on 31 queries by one f64 refinement against the f32 factor -- the
variance's share and, since round 6, the mean's (the residual y - m0 refined
the same way: alpha comes from the same inverse) -- and falls back to dgemm
products when either exceeds 5e-7.  Contract: mu and var within 1e-5
normwise of the fp64 oracle given the device factor (alpha solved in f64 from
it), under default options -- whichever sweep the probe picks.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402
from safe_bayesian_optimization_amd import TerrainMapper, synthetic  # noqa: E402
from safe_bayesian_optimization_amd import _native as N  # noqa: E402
from safe_bayesian_optimization_amd.terrain import Hyper, clustered, synthetic_box  # noqa: E402

REL_TOL = 1e-5
CHECK_TOL = 5e-7


@pytest.fixture(scope="module")
def mapper():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    O.set_threads(16)
    gm = TerrainMapper(0)
    yield gm
    gm.close()


def f32(a):
    return np.ascontiguousarray(a, np.float32)


def nrel(a, b):
    return float(np.abs(np.asarray(a, np.float64) - b).max() / max(np.abs(b).max(), 1e-30))


def oracle64(gm, wl):
    """fp64 posterior of the device's own f32 factor, alpha solved from it in f64."""
    from scipy.linalg import solve_triangular
    L, _ = gm.factor()
    o = gm.order()
    L64 = L.astype(np.float64)
    del L
    h = wl.hyper
    r = f32(wl.obs)[o].astype(np.float64) - h.prior_mean
    alpha = solve_triangular(L64.T, solve_triangular(L64, r, lower=True), lower=False)
    Lcm = O.colmajor_from_lower(L64)
    del L64
    return O.predict(Lcm, alpha, f32(wl.x)[o], f32(wl.y)[o], f32(wl.qx), f32(wl.qy), h.length_scale, h.sf2,
                     h.prior_mean)


def workload(n, box, hyper):
    """The domain and data of the default hyper-parameters (l = 0.4: the box,
    or a square of ~8 points per 0.4^2), fitted with `hyper` -- l = 1.6 there
    holds 128 points per l^2; a 32 x 16 query grid (the oracle costs N^2 per
    query)."""
    wl = synthetic_box(n, 32, 16, seed=n) if box else synthetic(n, 32, 16, seed=n + 5)
    wl.hyper = hyper
    return wl


CASES = [
    ("l1.6", 8192, False, Hyper(length_scale=1.6)),
    ("l1.6", 16384, False, Hyper(length_scale=1.6)),
    ("box_sn0.01", 8192, True, Hyper(noise_level=0.01)),
    ("box_sn0.01", 16384, True, Hyper(noise_level=0.01)),
    ("box_sn0.001", 16384, True, Hyper(noise_level=0.001)),
    ("box", 12288, True, Hyper()),
]


@pytest.mark.parametrize("name,n,box,hyper", CASES, ids=[f"{c[0]}-{c[1]}" for c in CASES])
def test_ill_conditioned_sliced_inverse(mapper, name, n, box, hyper):
    """Default options (six-digit sliced inverse, the guard on, the probe
    picking the sweep): the guard ran on the sliced inverse, and mu / var meet
    the contract against the oracle whatever it decided."""
    wl = workload(n, box, hyper)
    gm = TerrainMapper(0, hyper, ctx=mapper.ctx)
    gm.fit(wl.x, wl.y, wl.obs)
    chk = gm.inverse_check()
    precise, perr, _, _ = gm.precision()
    mu, sd = gm.predict(wl.qx, wl.qy)
    omu, ovar = oracle64(gm, wl)
    emu, evar = nrel(mu, omu), nrel(sd.astype(np.float64) ** 2, ovar)
    print(f"{name} n={n}: check err {chk['err']:.2e} (grid {chk['err_grid']:.2e} train {chk['err_train']:.2e}) "
          f"mean {chk['err_mean']:.2e} fired {chk['fired']} fallback {chk['err_fallback']:.2e} / "
          f"{chk['err_mean_fallback']:.2e} kept {chk['kept_digits']} {chk['ms']:.2f} ms; probe {perr:.2e} "
          f"precise {precise}; mu {emu:.2e} var {evar:.2e}")
    assert chk["ran"] == 1 and chk["digits"] == 6 and chk["m"] == 31
    assert chk["tol"] == CHECK_TOL
    passed = chk["err"] <= CHECK_TOL and chk["err_mean"] <= CHECK_TOL
    assert chk["fired"] == (0 if passed else 1)
    assert chk["kept_digits"] == (6 if passed else 0)
    if chk["fired"]:
        assert chk["err_fallback"] <= CHECK_TOL and chk["err_mean_fallback"] <= CHECK_TOL
    assert emu < REL_TOL and evar < REL_TOL


def test_guard_fires_on_five_digits(mapper):
    """SBO_OPT_INV_OZ = 5 on the lpsc box at N = 16384 moved the variance by
    3.7e-6 in round 4 (profiles/r4_inv_oz_ab.log): the guard must see it, redo
    the inverse with dgemm products (err_fallback: that inverse's own measure,
    orders below), and the posterior must then meet the contract; with the
    guard off the five-digit inverse stays and the posterior moves."""
    wl = workload(16384, True, Hyper())
    gm = TerrainMapper(0, wl.hyper, ctx=mapper.ctx)
    try:
        gm.set_option(N.SBO_OPT_INV_OZ, 5)
        gm.fit(wl.x, wl.y, wl.obs)
        chk = gm.inverse_check()
        mu, sd = gm.predict(wl.qx, wl.qy)
        omu, ovar = oracle64(gm, wl)
        emu, evar = nrel(mu, omu), nrel(sd.astype(np.float64) ** 2, ovar)
        print(f"five digits: check err {chk['err']:.2e} fired {chk['fired']} fallback {chk['err_fallback']:.2e} "
              f"{chk['ms']:.2f} ms; mu {emu:.2e} var {evar:.2e}")
        assert chk["ran"] == 1 and chk["digits"] == 5
        assert chk["err"] > CHECK_TOL and chk["fired"] == 1
        assert 0.0 <= chk["err_fallback"] < CHECK_TOL / 10
        assert emu < REL_TOL and evar < REL_TOL
        # the guard off: the five-digit inverse is kept (and is visibly worse)
        gm.set_option(N.SBO_OPT_INV_CHECK, 0)
        gm.fit(wl.x, wl.y, wl.obs)
        off = gm.inverse_check()
        assert off["ran"] == 0 and off["fired"] == 0
        mu5, sd5 = gm.predict(wl.qx, wl.qy)
        evar5 = nrel(sd5.astype(np.float64) ** 2, ovar)
        print(f"five digits, guard off: var {evar5:.2e}")
        assert evar5 > evar
    finally:
        gm.set_option(N.SBO_OPT_INV_OZ, 6)
        gm.set_option(N.SBO_OPT_INV_CHECK, 1)


def test_guard_sees_the_mean(mapper):
    """four digits on C4-like data move the whole-grid mean
    2.9e-6 while the variance reading stays 5e-8, inside the bound
    (profiles/r6_guard_mean.log) -- the round-5 guard kept that inverse.  The
    mean reading must see it (> 5e-7), the fit redo its inverse with dgemm
    products, and mu then meet the contract; with the guard off the
    four-digit mean stays and is visibly further from the oracle."""
    wl = synthetic(16384, 32, 16, seed=3)
    gm = TerrainMapper(0, wl.hyper, ctx=mapper.ctx)
    try:
        gm.set_option(N.SBO_OPT_INV_OZ, 4)
        gm.set_option(N.SBO_OPT_PRECISION, 1)      # (the precise sweep: the inverse's own effect shows)
        gm.fit(wl.x, wl.y, wl.obs)
        chk = gm.inverse_check()
        mu, sd = gm.predict(wl.qx, wl.qy)
        omu, ovar = oracle64(gm, wl)
        emu, evar = nrel(mu, omu), nrel(sd.astype(np.float64) ** 2, ovar)
        print(f"four digits: var reading {chk['err']:.2e} mean reading {chk['err_mean']:.2e} fired {chk['fired']} "
              f"kept {chk['kept_digits']} fallback {chk['err_fallback']:.2e} / {chk['err_mean_fallback']:.2e}; "
              f"mu {emu:.2e} var {evar:.2e}")
        assert chk["ran"] == 1 and chk["digits"] == 4
        assert chk["err"] <= CHECK_TOL < chk["err_mean"]     # the variance alone would have kept it
        assert chk["fired"] == 1 and chk["kept_digits"] == 0
        assert 0.0 <= chk["err_mean_fallback"] < CHECK_TOL / 100 and 0.0 <= chk["err_fallback"] < CHECK_TOL / 100
        assert emu < REL_TOL and evar < REL_TOL
        gm.set_option(N.SBO_OPT_INV_CHECK, 0)
        gm.fit(wl.x, wl.y, wl.obs)
        mu4, _ = gm.predict(wl.qx, wl.qy)
        emu4 = nrel(mu4, omu)
        print(f"four digits, guard off: mu {emu4:.2e}")
        assert emu4 > 10 * emu
    finally:
        gm.set_option(N.SBO_OPT_INV_OZ, 6)
        gm.set_option(N.SBO_OPT_INV_CHECK, 1)
        gm.set_option(N.SBO_OPT_PRECISION, -1)


def test_reduced_fit_on_clustered_same_area_data(mapper):
    """SBO_OPT_INV_OZ_ADAPT judges "the same data" by N, the
    hyper-parameters and the bounding box's area only, so clustered data in
    the same box (another conditioning) can follow a C4-like fit at five
    digits.  That reduced fit must read both the variance and the mean within
    tol / 8 or be redone at six digits -- either way mu and var meet the
    contract against the oracle."""
    n = 16384
    syn = synthetic(n, 32, 16, seed=3)
    cl = clustered(n, 32, 16, seed=7)
    gm = TerrainMapper(0, syn.hyper, ctx=mapper.ctx)
    first = []
    for _ in range(2):
        gm.fit(syn.x, syn.y, syn.obs)
        c = gm.inverse_check()
        first.append((c["digits"], f"{c['err']:.2e}", f"{c['err_mean']:.2e}", c["fired"]))
    print("C4-like fits:", first)
    assert first[1][0] == 5
    gm.fit(cl.x, cl.y, cl.obs)
    chk = gm.inverse_check()
    mu, sd = gm.predict(cl.qx, cl.qy)
    omu, ovar = oracle64(gm, cl)
    emu, evar = nrel(mu, omu), nrel(sd.astype(np.float64) ** 2, ovar)
    print(f"clustered after C4-like: digits {chk['digits']} var {chk['err']:.2e} mean {chk['err_mean']:.2e} "
          f"fired {chk['fired']} kept {chk['kept_digits']}; mu {emu:.2e} var {evar:.2e}")
    assert chk["digits"] == 5
    ok = chk["err"] <= CHECK_TOL / 8 and chk["err_mean"] <= CHECK_TOL / 8
    assert chk["fired"] == (0 if ok else 1) and chk["kept_digits"] == (5 if ok else 6)
    assert emu < REL_TOL and evar < REL_TOL


def test_guard_on_dgemm_inverse_and_appends(mapper):
    """SBO_OPT_INV_CHECK = 2 checks every full inverse: the dgemm one measures
    orders below the bound (the guard's own floor); with 1 and SBO_OPT_INV_OZ
    = 0 it does not run; appends keep the fit's result; below the slicing
    size (N <= 4096) the default does not run it."""
    wl = workload(8192, True, Hyper())
    gm = TerrainMapper(0, wl.hyper, ctx=mapper.ctx)
    try:
        gm.set_option(N.SBO_OPT_INV_OZ, 0)
        gm.set_option(N.SBO_OPT_INV_CHECK, 2)
        gm.fit(wl.x, wl.y, wl.obs)
        chk = gm.inverse_check()
        print(f"dgemm inverse: check err {chk['err']:.2e} {chk['ms']:.2f} ms")
        assert chk["ran"] == 1 and chk["digits"] == 0 and chk["fired"] == 0
        assert chk["err"] < CHECK_TOL / 100
        gm.set_option(N.SBO_OPT_INV_CHECK, 1)
        gm.fit(wl.x, wl.y, wl.obs)
        assert gm.inverse_check()["ran"] == 0
        gm.set_option(N.SBO_OPT_INV_OZ, 6)
        gm.fit(wl.x, wl.y, wl.obs)
        first = gm.inverse_check()
        assert first["ran"] == 1 and first["digits"] == 6
        extra = synthetic_box(8, 2, 2, seed=77)
        gm.append(extra.x, extra.y, extra.obs)
        assert gm.inverse_check() == first
        small = workload(4096, True, Hyper())
        gm.fit(small.x, small.y, small.obs)
        assert gm.inverse_check()["ran"] == 0
    finally:
        gm.set_option(N.SBO_OPT_INV_OZ, 6)
        gm.set_option(N.SBO_OPT_INV_CHECK, 1)
    with pytest.raises(N.SboError):
        gm.set_option(N.SBO_OPT_INV_CHECK, 3)


def test_inverse_digits_adapt(mapper):
    """SBO_OPT_INV_OZ_ADAPT (default): a refit of the same hyper-parameters and
    about the same N takes five digits when the last guard readings (variance
    and mean) predict them within an eighth of the bound (C4-like synthetic
    data: 1.4e-12 / 1.2e-10 at six),
    and its posterior -- the precise sweep, so that the inverse's own effect
    shows -- stays within 2e-7 of the six-digit fit's and meets the contract;
    the lpsc box (3.8e-9 at six) stays at six, and after the synthetic data
    its different box area (density) makes it new data; a changed
    hyper-parameter, N or box, or an option change, start again at six.  (A
    reduced fit that fires pins its data to six digits:
    test_diagnostic_only_variants forces five digits on the box through the
    diagnostic build.)"""
    n = 16384
    syn = synthetic(n, 32, 16, seed=3)
    box = synthetic_box(n, 32, 16, seed=3)
    gm = TerrainMapper(0, syn.hyper, ctx=mapper.ctx)
    try:
        gm.set_option(N.SBO_OPT_INV_OZ_ADAPT, 1)
        gm.set_option(N.SBO_OPT_PRECISION, 1)
        got = []
        for _ in range(3):
            gm.fit(syn.x, syn.y, syn.obs)
            c = gm.inverse_check()
            mu, sd = gm.predict(syn.qx, syn.qy)
            got.append((c, mu.astype(np.float64), sd.astype(np.float64) ** 2))
        print("synthetic:", [(c["digits"], f"{c['err']:.1e}", c["fired"]) for c, _, _ in got])
        assert [c["digits"] for c, _, _ in got] == [6, 5, 5]
        assert all(c["fired"] == 0 and c["err"] <= CHECK_TOL / 100 and c["err_mean"] <= CHECK_TOL / 8
                   for c, _, _ in got)
        dmu, dvar = nrel(got[2][1], got[0][1]), nrel(got[2][2], got[0][2])
        print(f"five vs six digits: mu {dmu:.2e} var {dvar:.2e}")
        assert dmu < 2e-7 and dvar < 2e-7
        omu, ovar = oracle64(gm, syn)
        assert nrel(got[2][1], omu) < REL_TOL and nrel(got[2][2], ovar) < REL_TOL
        # the lpsc box: the same N and hyper-parameters but 1/130 of the area
        # (another density): not the same data, six digits
        gm.fit(box.x, box.y, box.obs)
        assert gm.inverse_check()["digits"] == 6
        gm.fit(syn.x, syn.y, syn.obs)
        assert gm.inverse_check()["digits"] == 6
        gm.fit(syn.x, syn.y, syn.obs)
        assert gm.inverse_check()["digits"] == 5
        # new data (another N): six, then five again; an option change: six
        syn2 = synthetic(12288, 32, 16, seed=9)
        ds = []
        for k in range(3):
            if k == 2:
                gm.set_option(N.SBO_OPT_INV_OZ, 6)
            gm.fit(syn2.x, syn2.y, syn2.obs)
            ds.append(gm.inverse_check()["digits"])
        assert ds == [6, 5, 6]
        # another hyper-parameter: six
        gm.fit(syn2.x, syn2.y, syn2.obs)
        assert gm.inverse_check()["digits"] == 5
        gm2 = TerrainMapper(0, Hyper(length_scale=0.41), ctx=mapper.ctx)
        gm2.fit(syn2.x, syn2.y, syn2.obs)
        assert gm2.inverse_check()["digits"] == 6
        # the lpsc box stays at six; adaptation off: always six
        gm.set_option(N.SBO_OPT_INV_OZ_ADAPT, 0)
        gm.fit(syn.x, syn.y, syn.obs)
        gm.fit(syn.x, syn.y, syn.obs)
        assert gm.inverse_check()["digits"] == 6
        gm.set_option(N.SBO_OPT_INV_OZ_ADAPT, 1)
        bx = workload(16384, True, Hyper())
        for _ in range(2):
            gm.fit(bx.x, bx.y, bx.obs)
            assert gm.inverse_check()["digits"] == 6
    finally:
        gm.set_option(N.SBO_OPT_PRECISION, -1)
        gm.set_option(N.SBO_OPT_INV_OZ_ADAPT, 1)
    with pytest.raises(N.SboError):
        gm.set_option(N.SBO_OPT_INV_OZ_ADAPT, 2)
